"""HBM bandwidth reference points on the headline's tensor sizes (fp32 [6.55 M px][64 ch] = 1.68 GB): write-only
(fill), read-only (sum), copy (read + write) and a 1:4 read:write mix, in TB/s of bytes moved."""
import json

import torch


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    n = 6553600 * 64
    a = torch.empty(n, device="cuda")
    b = torch.empty(n, device="cuda")
    q = torch.empty(n // 4, device="cuda").normal_()
    a.normal_()
    gb = n * 4 / 1e9
    res = {"fill_TBs": gb / timeit(lambda: a.fill_(1.0)) / 1e3,
           "sum_TBs": gb / timeit(lambda: a.sum()) / 1e3,
           "copy_TBs": 2 * gb / timeit(lambda: b.copy_(a)) / 1e3,
           "expand_1to4_TBs": 1.25 * gb / timeit(lambda: b.view(-1, 4).copy_(q.view(-1, 1).expand(-1, 4))) / 1e3}
    print(json.dumps({k: round(v, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()

"""Diagnostic: leave non-zero data in freed device memory (a large random fill released back to the driver), then run
the 8-rank deterministic-equality rehearsal in fresh processes — if it then fails where it passes on a clean card,
some kernel reads device memory it never wrote."""
import subprocess
import sys

import torch


def main():
    free, _ = torch.cuda.mem_get_info()
    n = int(free * 0.6) // 4
    x = torch.empty(n, device="cuda")
    x.uniform_(-1.0, 1.0)
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()
    print(f"filled and released {n * 4 / 2**30:.1f} GiB", flush=True)
    rc = subprocess.call([sys.executable, "-u", "-m", "pytest", "-q", "--timeout", "600", "--timeout-method", "thread",
                          "-p", "no:cacheprovider",
                          "tests/test_rccl_dist_gpu.py::test_headline_config_eight_ranks_ragged_packing_equals_one_rank"])
    sys.exit(rc)


if __name__ == "__main__":
    main()

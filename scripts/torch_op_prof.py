#!/usr/bin/env python3
"""Which PyTorch ops launch the non-native ("at::native") kernels of a bench preset: runs bench.py's
configuration with the timed rounds under torch.profiler (HIP graphs off, so every kernel is attributed to
the op that launched it) and prints the ops by self device time.

    FEDML_AMD_HIP_GRAPHS=0 python scripts/torch_op_prof.py --preset distilbert_fedopt_32 [--rows 40]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="distilbert_fedopt_32")
    ap.add_argument("--rows", type=int, default=40)
    ap.add_argument("--trace-dtoh", action="store_true")
    ap.add_argument("--trace-big", action="store_true")
    ap.add_argument("--shapes", default="", help="ops whose input shapes are printed (comma list)")
    ap.add_argument("--stacks", default="aten::copy_,aten::fill_,aten::add_,aten::add,aten::zero_,aten::mul",
                    help="ops whose Python call sites are printed (comma list; '' = none)")
    a, rest = ap.parse_known_args()
    import torch
    import bench
    from fedml_amd.simulation.rccl import simulator as S
    orig = S.RCCLSimulator.run
    state = {"n": 0}

    def run(self, n):
        state["n"] += 1
        if state["n"] == 1:        # warmup round (bench --warmup 1)
            return orig(self, n)
        acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
        with torch.profiler.profile(activities=acts, with_stack=bool(a.stacks), record_shapes=bool(a.shapes)) as prof:
            r = orig(self, n)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60),
              flush=True)
        if a.shapes:   # the input shapes of the listed ops, by device time
            want_s = set(a.shapes.split(","))
            rows_s = [e for e in prof.key_averages(group_by_input_shape=True) if e.key in want_s]
            def dev_t_(e):
                return getattr(e, "self_device_time_total", 0.0) or getattr(e, "self_cuda_time_total", 0.0)

            rows_s.sort(key=lambda e: -dev_t_(e))
            for e in rows_s[:20]:
                dev_t = dev_t_(e)
                print(f"== {e.key} calls {e.count} self device {dev_t / 1e3:.2f} ms shapes {e.input_shapes}")
        if a.stacks:
            want = set(a.stacks.split(","))
            rows = [e for e in prof.key_averages(group_by_stack_n=8) if e.key in want]
            def dev_us(e):
                return getattr(e, "self_device_time_total", None) or getattr(e, "self_cuda_time_total", 0.0)

            rows.sort(key=lambda e: -dev_us(e))
            for e in rows[:25]:
                print(f"== {e.key}  calls {e.count}  self device {dev_us(e) / 1e3:.2f} ms")
                for fr in e.stack[:8]:
                    print("     ", fr)
        return r

    S.RCCLSimulator.run = run
    if a.trace_dtoh:   # print the Python call site of every device→host copy above 1 MB
        import traceback
        seen = {}

        def wrap(name):
            orig_m = getattr(torch.Tensor, name)

            def f(t, *args, **kw):
                if t.is_cuda and t.numel() * t.element_size() > (1 << 20):
                    dst = args[0] if args else kw.get("device", kw.get("dtype"))
                    if name != "to" or (isinstance(dst, (str, torch.device)) and str(dst).startswith("cpu")):
                        site = "".join(traceback.format_stack(limit=6)[:-1])
                        seen[site] = seen.get(site, 0) + 1
                        if seen[site] == 1:
                            print(f"== DtoH via Tensor.{name}: {t.numel() * t.element_size() / 2**20:.1f} MB\n{site}",
                                  flush=True)
                return orig_m(t, *args, **kw)
            setattr(torch.Tensor, name, f)
        for n_ in ("cpu", "to", "numpy", "tolist", "item"):
            wrap(n_)
    if a.trace_big:    # print the Python call site of every in-place copy_/fill_/zero_ on a tensor above 64 MB
        import traceback
        seen_b = {}

        def wrap_b(name):
            orig_m = getattr(torch.Tensor, name)

            def f(t, *args, **kw):
                if t.is_cuda and t.numel() * t.element_size() > (64 << 20):
                    site = "".join(traceback.format_stack()[-8:-1])
                    seen_b[site] = seen_b.get(site, 0) + 1
                    if seen_b[site] == 1:
                        print(f"== Tensor.{name} on {t.numel() * t.element_size() / 2**20:.0f} MB "
                              f"(contiguous {t.is_contiguous()})\n{site}", flush=True)
                return orig_m(t, *args, **kw)
            setattr(torch.Tensor, name, f)
        for n_ in ("copy_", "fill_", "zero_"):
            wrap_b(n_)
    sys.argv = ["bench.py", "--preset", a.preset, "--steps", "1", "--warmup", "1"] + rest
    bench.main()


if __name__ == "__main__":
    main()

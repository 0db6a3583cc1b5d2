"""Deterministic-mode reproducibility probe: the same multi-process RCCL-simulator run (tests/dist_worker_rccl_sim.py)
several times; prints whether every repeat is bitwise equal to the first, per world size.

    python scripts/det_repro.py --model headline --clients 100 --worlds 1,8 --repeats 3 --rounds 2
"""
import argparse
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="headline")
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--worlds", default="1,8")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--rounds", default="2")
    ap.add_argument("--shuffle", type=int, default=1)
    ap.add_argument("--augment", type=int, default=0)
    a = ap.parse_args()
    import torch
    from test_rccl_dist import _launch
    env = dict(FEDML_TEST_DEVICE="cuda", FEDML_AMD_DIST_BACKEND="gloo", FEDML_TEST_ROUNDS=a.rounds,
               HSA_ENABLE_IPC_MODE_LEGACY="0", FEDML_AMD_DETERMINISTIC="1")
    ref = {}
    with tempfile.TemporaryDirectory() as td:
        for wsz in [int(v) for v in a.worlds.split(",")]:
            runs = []
            for r in range(a.repeats):
                w = _launch(wsz, os.path.join(td, f"w{wsz}_{r}.pt"), a.model, a.clients, bool(a.shuffle),
                            bool(a.augment), **env)
                runs.append(w)
                same = torch.equal(w, runs[0])
                nd = int((w != runs[0]).sum())
                print(f"world {wsz} repeat {r}: equal to repeat 0: {same} (differing elements {nd}, rel "
                      f"{float((w - runs[0]).norm() / runs[0].norm()):.3e})", flush=True)
            ref[wsz] = runs[0]
        ws = sorted(ref)
        for wsz in ws[1:]:
            print(f"world {wsz} vs world {ws[0]}: equal {torch.equal(ref[wsz], ref[ws[0]])}, differing elements "
                  f"{int((ref[wsz] != ref[ws[0]]).sum())}", flush=True)


if __name__ == "__main__":
    main()

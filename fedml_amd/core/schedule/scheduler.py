"""Client → GPU workload scheduler (D5).

The reference ships a branch-and-bound scheduler that nothing calls
(`core/schedule/scheduler.py:4-172`). Here it is native
(``csrc/runtime.cpp::fr_schedule``: best-first search with a node budget and
an LPT completion) and it is *used*: the RCCL simulator calls
``pack_clients_to_gpus`` to decide which virtual clients each MI355X hosts.
"""
import ctypes

import numpy as np

from ...utils.native_runtime import runtime_lib


def _schedule_py(workloads, mem, speed, memory, mode, node_budget):
    # pure-python LPT fallback (used only if the native lib cannot be built)
    n, m = len(workloads), len(speed)
    order = np.argsort(-np.asarray(workloads), kind="stable")
    cost = np.zeros(m)
    res = np.zeros(m)
    assign = np.full(n, -1, dtype=np.int32)
    for w in order:
        best, best_c = -1, None
        for j in range(m):
            nm = res[j] + mem[w] if mode == 1 else max(res[j], mem[w])
            if nm > memory[j]:
                continue
            c = cost[j] + speed[j] * workloads[w]
            if best < 0 or c < best_c:
                best, best_c = j, c
        if best < 0:
            return -1.0, assign
        cost[best] = best_c
        res[best] = res[best] + mem[w] if mode == 1 else max(res[best], mem[w])
        assign[w] = best
    return float(cost.max()), assign


class Scheduler:
    def __init__(self, workloads, constraints, memory, mem_per_workload=None):
        self.workloads = np.asarray(workloads, dtype=np.float64)
        self.speed = np.asarray(constraints, dtype=np.float64)
        self.memory = np.asarray(memory, dtype=np.float64)
        self.mem_per_wl = (np.asarray(mem_per_workload, dtype=np.float64)
                           if mem_per_workload is not None else self.workloads.copy())

    def assign(self, mode=1, node_budget=200000):
        n, m = len(self.workloads), len(self.speed)
        lib = runtime_lib()
        if lib is None:
            return _schedule_py(self.workloads, self.mem_per_wl, self.speed, self.memory, mode, node_budget)
        out = np.full(n, -1, dtype=np.int32)
        cost = lib.fr_schedule(
            n, self.workloads.ctypes.data_as(ctypes.c_void_p), self.mem_per_wl.ctypes.data_as(ctypes.c_void_p),
            m, self.speed.ctypes.data_as(ctypes.c_void_p), self.memory.ctypes.data_as(ctypes.c_void_p),
            int(mode), int(node_budget), out.ctypes.data_as(ctypes.c_void_p))
        return float(cost), out

    def DP_schedule(self, mode=1):
        """Reference-shaped output: per resource, a dict {bunch_idx: [workload indices]} where a
        bunch is a set of clients resident at the same time (mode 1) or one client (mode 0)."""
        cost, assign = self.assign(mode)
        if cost < 0:
            raise RuntimeError("no feasible schedule under the memory constraints")
        out = []
        for j in range(len(self.speed)):
            jobs = [int(i) for i in np.argsort(-self.workloads, kind="stable") if assign[i] == j]
            sched = {}
            if mode == 1:
                cur, foot = [], 0.0
                for i in jobs:
                    if foot + self.mem_per_wl[i] <= self.memory[j]:
                        cur.append(i)
                        foot += self.mem_per_wl[i]
                    else:
                        sched[len(sched)] = cur
                        cur, foot = [i], self.mem_per_wl[i]
                if cur:
                    sched[len(sched)] = cur
            else:
                for i in jobs:
                    sched[len(sched)] = [i]
            out.append(sched)
        self.makespan = cost
        return out


# reference spelling
scheduler = Scheduler


def _lpt_balanced(counts, n_gpus, speed, cap):
    """Longest-processing-time greedy under a per-GPU client cap: O(C log C), within 4/3 of the
    optimum makespan (Graham) — the per-round path, where the branch-and-bound's tens of ms per
    round would be serial host time on every rank."""
    order = sorted(range(len(counts)), key=lambda i: (-counts[i], i))
    load = [0.0] * n_gpus
    n = [0] * n_gpus
    out = [[] for _ in range(n_gpus)]
    for i in order:
        best = min((g for g in range(n_gpus) if n[g] < cap[g]), key=lambda g: ((load[g] + counts[i]) / speed[g], g))
        out[best].append(i)
        load[best] += counts[i]
        n[best] += 1
    return [sorted(o) for o in out]


_PACK_CACHE = {}


def pack_clients_to_gpus(sample_counts, n_gpus, gpu_speed=None, gpu_mem_bytes=None, bytes_per_client=0.0,
                         balance_counts=True, exact=False):
    """Assign clients to GPUs minimising the max per-GPU work (samples × speed).

    With ``balance_counts`` the assignment is additionally constrained to give each GPU
    ⌈C/G⌉ or ⌊C/G⌋ clients (the batched engine steps all resident clients together, so a
    GPU's step count is set by its largest client and the number of clients it hosts);
    inside that constraint the native branch-and-bound balances total samples.
    Returns a list of client-index lists, one per GPU.
    """
    c = len(sample_counts)
    # Per-round fast paths (the simulator packs every round on every rank): equal counts → contiguous
    # balanced chunks; otherwise the LPT greedy, memoised per (counts, GPUs). ``exact`` runs the
    # native branch-and-bound (fr_schedule) instead.
    if balance_counts and gpu_mem_bytes is None and not exact:
        counts = [float(v) for v in sample_counts]
        sp = [1.0] * n_gpus if gpu_speed is None else [float(v) for v in gpu_speed]
        key = (tuple(counts), n_gpus, tuple(sp))
        hit = _PACK_CACHE.get(key)
        if hit is not None:
            return [list(v) for v in hit]
        if len(set(counts)) <= 1 and len(set(sp)) <= 1:
            q, r = divmod(c, n_gpus)
            out, lo = [], 0
            for g in range(n_gpus):
                hi = lo + q + (1 if g < r else 0)
                out.append(list(range(lo, hi)))
                lo = hi
        else:
            cap = [int(np.ceil(c / n_gpus))] * n_gpus
            out = _lpt_balanced(counts, n_gpus, sp, cap)
        if len(_PACK_CACHE) > 4096:
            _PACK_CACHE.clear()
        _PACK_CACHE[key] = [tuple(v) for v in out]
        return out
    speed = np.ones(n_gpus) if gpu_speed is None else np.asarray(gpu_speed, dtype=np.float64)
    if gpu_mem_bytes is None:
        mem = np.full(n_gpus, np.inf)
    else:
        mem = np.asarray(gpu_mem_bytes, dtype=np.float64)
    if balance_counts:
        # memory budget expressed in "client slots" enforces the count balance
        cap = int(np.ceil(c / n_gpus))
        slots = np.full(n_gpus, float(cap))
        if gpu_mem_bytes is not None and bytes_per_client > 0:
            slots = np.minimum(slots, np.floor(mem / bytes_per_client))
        sch = Scheduler(np.asarray(sample_counts, dtype=np.float64), speed, slots, np.ones(c))
    else:
        sch = Scheduler(np.asarray(sample_counts, dtype=np.float64), speed, mem,
                        np.full(c, float(bytes_per_client)))
    cost, assign = sch.assign(mode=1, node_budget=20000)
    if cost < 0:
        raise RuntimeError("client packing infeasible: not enough GPU memory for the resident clients")
    return [sorted(int(i) for i in np.where(assign == j)[0]) for j in range(n_gpus)]

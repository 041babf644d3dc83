"""Project bench.py's strong scaling over 1/2/4/8 GPUs from one GPU's measured per-problem solve times.

Input: tools/tail_probe.py's npz (every problem of config D solved once in one launch: cycles per problem,
i.e. the wavefront time of that solve at full load).  Model of bench.py: the global batch GB = 32768 is solved
`steps` times; the step-major ticket list is cut into chunks of 256 (multi-GPU) and the ranks start on contiguous
shares and steal tail chunks (scheduler.py); every GPU runs 1 024 wavefronts that claim tickets in order.
Two brackets:
  * ideal stealing: tickets list-scheduled in order over all N x 1 024 wavefronts (a wave takes the next ticket
    the moment it is free, on whichever GPU);
  * chunked stealing: chunks list-scheduled over the GPUs by their predicted finish time, then each GPU's tickets
    list-scheduled over its 1 024 waves (what the steal plan approximates).
Efficiency(N) = T(1) / (N T(N)); solves/s(N) = steps GB / T(N) with the 1-GPU rate calibrated to the probe's
cycles per ms.  Per-iteration time is taken as load-independent (each GPU stays full while it has tickets).

    python tools/scale_projection.py profiles/r04_tail_D.npz [steps ...] > profiles/r04_scale_projection.json
"""
import heapq
import json
import sys

import numpy as np


def list_schedule(durations, workers):
    free = [0.0] * workers
    heapq.heapify(free)
    for d in durations:
        heapq.heappush(free, heapq.heappop(free) + d)
    return max(free)


def chunked(durations, gpus, waves, chunk=256):
    if gpus == 1:
        return list_schedule(durations, waves)
    chunks = [durations[i:i + chunk] for i in range(0, len(durations), chunk)]
    # greedy: each chunk to the GPU with the least assigned work (what steals converge to), in ticket order
    loads = [0.0] * gpus
    per = [[] for _ in range(gpus)]
    for c in chunks:
        g = int(np.argmin(loads))
        per[g].extend(c)
        loads[g] += float(np.sum(c)) / waves
    return max(list_schedule(p, waves) for p in per)


def main():
    z = np.load(sys.argv[1])
    steps_list = [int(v) for v in sys.argv[2:]] or [6, 20]
    cyc = z["cycles"].astype(np.float64)
    waves = int(z["waves"])
    cpm = float(z["cycles_per_ms"])
    GB = len(cyc)
    out = {"source": sys.argv[1], "global_batch": GB, "waves_per_gpu": waves, "cycles_per_ms": cpm,
           "mean_iterations": float(np.mean(z["iterations"])), "max_iterations": int(np.max(z["iterations"])),
           "longest_solve_ms": float(cyc.max() / cpm), "projections": []}
    for steps in steps_list:
        tickets = np.tile(cyc, steps)
        base = None
        for n in (1, 2, 4, 8):
            ideal = list_schedule(tickets, n * waves) / cpm
            ch = chunked(tickets, n, waves) / cpm
            if base is None:
                base = ideal
            out["projections"].append({
                "steps": steps, "gpus": n,
                "ideal_ms": ideal, "chunked_ms": ch,
                "solves_per_s_ideal": steps * GB / (ideal / 1e3), "solves_per_s_chunked": steps * GB / (ch / 1e3),
                "efficiency_ideal": base / (n * ideal), "efficiency_chunked": base / (n * ch),
                "work_over_capacity_ms": float(tickets.sum() / (n * waves) / cpm)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

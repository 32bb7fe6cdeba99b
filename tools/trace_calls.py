#!/usr/bin/env python3
"""Per-launch kernel durations from a rocprofv3 kernel trace of `bench.py` (diagnostic).

bench.py's time_kernels() queues every C-ABI call of the step behind a spin kernel, 20 times.
This groups the trace into (spin, kernels of one call) segments and prints, per call of the
step, the median duration of each kernel it launched and the gap to the next kernel.

    python3 tools/trace_calls.py gpurun_out/PROF/run_kernel_trace.csv [--reps 20]
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--reps" else 20
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "spin_kernel" in name:
            if cur is not None:
                segs.append(cur)
            cur = []
            continue
        if cur is not None:
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r))
    if cur:
        segs.append(cur)
    # the isolated section is the last ncalls*reps segments
    ncalls = len(segs) // reps
    segs = segs[-ncalls * reps:]
    total = 0.0
    for c in range(ncalls):
        group = segs[c * reps:(c + 1) * reps]
        nk = len(group[0])
        parts = []
        for k in range(nk):
            durs = [(g[k][2] - g[k][1]) / 1e3 for g in group if len(g) == nk]
            gaps = [(g[k + 1][1] - g[k][2]) / 1e3 for g in group if len(g) == nk and k + 1 < nk]
            name = group[0][k][0]
            short = name.split("(")[0].replace("void ", "")[-70:]
            r = group[0][k][3]
            med = statistics.median(durs)
            total += med
            parts.append(f"{short} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} "
                         f"vgpr={r['VGPR_Count']}+{r['Accum_VGPR_Count']} lds={r['LDS_Block_Size']} "
                         f"{med:.2f}us" + (f" gap {statistics.median(gaps):.2f}" if gaps else ""))
        print(f"[{c:2d}] " + " | ".join(parts))
    print(f"sum of kernel medians: {total:.1f} us")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Print a kprobe JSON (tools/kprobe.py) as a table: per launch the blocks, span and the median
per-block phase durations (us)."""
import json
import sys

rows = json.load(open(sys.argv[1]))
print(f"{'#':>3} {'fn':26s} {'blk':>5} {'span':>6} {'skew':>5} {'bmed':>6} {'ph1':>5} {'ph2':>5} {'ph3':>5} {'ph3max':>6}")
for r in rows:
    if r.get('blocks', 0) == 0:
        continue
    print(f"{r['launch']:3d} {r['fn']:26s} {r['blocks']:5d} {r['span_us']:6.2f} {r['start_skew_us']:5.2f} "
          f"{r['block_us_med']:6.2f} {r['prologue_med']:5.2f} {r['loop_med']:5.2f} {r['epilogue_med']:5.2f} {r['epilogue_max']:6.2f}")

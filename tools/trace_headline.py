"""Per-leg launch statistics of the bench's kernel trace (rocprofv3 --kernel-trace): the headline
kernel's name also runs the cold-cache and 2^22 legs, so the --stats summary mixes them; this splits
the trace by kernel name and grid size, in launch order, and reports the headline's timed launches
(the 50 after the 10 warm-ups) on their own.
    python tools/trace_headline.py gpurun_out/prof/bench/bench_kernel_trace.csv > profiles/r02_bench_trace_legs.json"""
import collections
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
warm, steps = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (10, 50)
legs = collections.OrderedDict()
for r in rows:
    if r["Kernel_Name"].startswith("kinhip"):
        legs.setdefault((r["Kernel_Name"], int(r["Grid_Size_X"])), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {"source": sys.argv[1], "legs": []}
for (name, grid), d in legs.items():
    out["legs"].append({"kernel": name, "grid_threads": grid, "launches": len(d), "avg_us": sum(d) / len(d),
                        "min_us": min(d), "max_us": max(d)})
head = next(((k, d) for k, d in legs.items() if k[0].startswith("kinhip_jit_fk_f32") and k[1] == 1 << 20), None)
if head:
    timed = head[1][warm:warm + steps]
    out["headline"] = {"kernel": head[0][0], "grid_threads": head[0][1], "warmup": warm, "timed_launches": len(timed),
                       "avg_us": sum(timed) / len(timed), "min_us": min(timed), "max_us": max(timed),
                       "later_launches_of_this_name_and_grid": len(head[1]) - warm - steps,
                       "note": "the later launches are the cold-cache leg (1 + 10 launches after a 1 GiB read)"}
print(json.dumps(out, indent=1))

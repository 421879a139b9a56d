"""Summarise rocprofv3 --pmc passes of the matcher (tools/gpu_pmc.sh) into one JSON under
profiles/: per-launch averages, HBM bytes = 2*FETCH_SIZE*1024 (gfx950 reports half of a
wide coalesced stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE*1024, the effective clock
GRBM_GUI_ACTIVE/8/t and the MFMA-busy fraction.
    python tools/pmc_summary.py gpurun_out/pmc_<kernel>_c3 profiles/r01_pmc_<kernel>_c3.json \
        <kernel_ms> <kernel>"""
import collections
import csv
import json
import os
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
kernel_ms = float(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "-" else None
kernel = sys.argv[4] if len(sys.argv) > 4 else "match_i8_kernel"
vals = collections.defaultdict(list)
gui_clock = []   # per dispatch of the pass that holds GRBM_GUI_ACTIVE: cycles / its own duration
for sub in sorted(os.listdir(src)):
    f = os.path.join(src, sub, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        if re.search(r"(^|::|\s)%s\b" % kernel, r["Kernel_Name"]):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp"):
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                if dur > 0:
                    gui_clock.append(float(r["Counter_Value"]) / 8 / dur / 1e9)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
out = {"kernel": kernel, "counters_per_launch": avg}
if gui_clock:   # the profiled dispatches' own clock (MI355X_MICROARCH.md, DVFS)
    out["clock_ghz_profiled"] = sum(gui_clock) / len(gui_clock)
if "FETCH_SIZE" in avg:
    out["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
if "WRITE_SIZE" in avg:
    out["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
if "hbm_read_bytes" in out and "hbm_write_bytes" in out:
    out["hbm_bytes"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
if kernel_ms and "GRBM_GUI_ACTIVE" in avg:
    cyc = avg["GRBM_GUI_ACTIVE"] / 8
    out["kernel_ms"] = kernel_ms
    out["clock_ghz"] = cyc / (kernel_ms * 1e-3) / 1e9
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        out["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))

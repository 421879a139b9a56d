"""Summarise rocprofv3 --pmc passes of the matcher (tools/gpu_pmc.sh) into one JSON under
profiles/: per-launch averages, HBM bytes = 2*FETCH_SIZE*1024 (gfx950 reports half of a
wide coalesced stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE*1024, the effective clock
GRBM_GUI_ACTIVE/8 over each profiled dispatch's own duration and the MFMA-busy fraction.
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
    c = sum(gui_clock) / len(gui_clock)
    if c <= 2.4:
        out["clock_ghz_profiled"] = c
    else:
        # GRBM_GUI_ACTIVE spans a little more than the dispatch's own timestamps: on short
        # dispatches (one query image, ~70 us) the ratio exceeds the chip's 2.4 GHz, so it
        # is no clock measurement there
        out["clock_ghz_profiled"] = None
        out["clock_note"] = ("GRBM_GUI_ACTIVE/8 over the dispatch duration = %.3f GHz > 2.4: the "
                             "counter window exceeds a short dispatch; not a clock" % c)
if "FETCH_SIZE" in avg:
    out["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
if "WRITE_SIZE" in avg:
    out["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
if "hbm_read_bytes" in out and "hbm_write_bytes" in out:
    out["hbm_bytes"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
if "GRBM_GUI_ACTIVE" in avg:
    # the clock is the profiled dispatches' own (cycles over their own duration, above);
    # dividing their cycles by an UNprofiled launch time (rounds 1-3) mixed two runs and gave
    # clocks above the chip's 2.4 GHz
    cyc = avg["GRBM_GUI_ACTIVE"] / 8
    if kernel_ms:
        out["kernel_ms_unprofiled"] = kernel_ms
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        out["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))

"""Per-image SIFT timeline from a rocprofv3 kernel trace of tools/sift_prof.py: kernels
grouped per image (an image starts at upscale_kernel), per-kernel time per image, and for
the last images the wall span, the busy union and the idle gaps between kernels.
    python tools/sift_timeline.py <kernel_trace.csv> <images timed>"""
import collections
import csv
import re
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"::(\w+?)(<[^>]*>)?\(", r["Kernel_Name"])
    name = m.group(1) + (m.group(2) or "") if m else r["Kernel_Name"][:40]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
images, cur = [], []
for s, e, n in rows:
    if n.startswith("upscale_kernel") and cur:
        images.append(cur)
        cur = []
    cur.append((s, e, n))
if cur:
    images.append(cur)
nimg = int(sys.argv[2]) if len(sys.argv) > 2 else 10
last = [im for im in images if any(n.startswith("descriptor_kernel") for _, _, n in im)][-nimg:]
per = collections.defaultdict(float)
cnt = collections.Counter()
for im in last:
    for s, e, n in im:
        per[n] += (e - s) / 1e3
        cnt[n] += 1
print("kernels per image (us, launches):")
for n, t in sorted(per.items(), key=lambda kv: -kv[1]):
    print("  %-44s %8.1f  %4.1f" % (n[:44], t / len(last), cnt[n] / len(last)))
print("  %-44s %8.1f" % ("sum", sum(per.values()) / len(last)))
spans, busy = [], []
for im in last:
    t0 = im[0][0]
    t1 = max(e for _, e, _ in im)
    spans.append((t1 - t0) / 1e3)
    # busy union
    iv = sorted((s, e) for s, e, _ in im)
    u, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            u += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    u += ce - cs
    busy.append(u / 1e3)
print("span first kernel -> last end: %.1f us (min %.1f), busy union %.1f us" %
      (sum(spans) / len(spans), min(spans), sum(busy) / len(busy)))
im = last[-1]
t0 = im[0][0]
print("last image, kernel by kernel (start, dur, gap before, us):")
pe = t0
for s, e, n in im:
    print("  %8.1f %7.1f %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - pe) / 1e3, n[:50]))
    pe = max(pe, e)

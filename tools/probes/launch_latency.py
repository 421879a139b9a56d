import csv, glob, sys, numpy as np
d = sys.argv[1]
k = list(csv.DictReader(open(glob.glob(d + '/*kernel_trace.csv')[0])))
a = list(csv.DictReader(open(glob.glob(d + '/*hip_api_trace.csv')[0])))
api = {int(r['Correlation_Id']): r for r in a}
lat = []
for r in k:
    c = int(r['Correlation_Id'])
    if c in api and api[c]['Function'] in ('hipLaunchKernel', 'hipExtLaunchKernel'):
        lat.append((int(r['Start_Timestamp']) - int(api[c]['Start_Timestamp'])) / 1e3)
lat = np.array(lat)
print('launch call -> kernel start: n %d, median %.1f us, p10 %.1f, p90 %.1f' % (len(lat), np.median(lat), np.percentile(lat, 10), np.percentile(lat, 90)))
# first launch after an idle gap (> 100 us since the previous kernel's end)
ks = sorted(k, key=lambda r: int(r['Start_Timestamp']))
first = []
prev_end = None
for r in ks:
    c = int(r['Correlation_Id'])
    s = int(r['Start_Timestamp'])
    if prev_end is not None and s - prev_end > 100000 and c in api:
        first.append((s - int(api[c]['Start_Timestamp'])) / 1e3)
    prev_end = int(r['End_Timestamp'])
first = np.array(first)
if len(first):
    print('first launch after idle: n %d, median %.1f us, p10 %.1f, p90 %.1f' % (len(first), np.median(first), np.percentile(first, 10), np.percentile(first, 90)))

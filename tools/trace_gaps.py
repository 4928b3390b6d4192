#!/usr/bin/env python3
"""Gaps between consecutive coding launches in a rocprofv3 --kernel-trace
--memory-copy-trace directory (tools/gpu_session.sh profcopy), and where the
last table copy ended relative to each launch.  python tools/trace_gaps.py DIR"""
import csv, sys, statistics
d = sys.argv[1]
ks = [r for r in csv.DictReader(open(d + '/run_kernel_trace.csv')) if 'gf8' in r['Kernel_Name'] or 'expand' in r['Kernel_Name']]
cs = list(csv.DictReader(open(d + '/run_memory_copy_trace.csv')))
ev = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K' if 'gf8' in r['Kernel_Name'] else 'X') for r in ks]
ev += [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C') for r in cs]
ev.sort()
g = [e for e in ev if e[2] == 'K']
gaps = [g[i + 1][0] - g[i][1] for i in range(len(g) - 1)]
print('kernels', len(g), 'gap us median %.1f min %.1f max %.1f' % (statistics.median(gaps) / 1e3, min(gaps) / 1e3, max(gaps) / 1e3))
# relation of copy end to next kernel start
for i in range(20, 24):
    s, e, k = g[i]
    prev_c = [c for c in ev if c[2] == 'C' and c[1] <= s]
    c = prev_c[-1] if prev_c else None
    print('k%d dur %.1f us, gap before %.1f us, last copy ended %.1f us before start (copy %.1f us)' % (
        i, (e - s) / 1e3, (s - g[i - 1][1]) / 1e3, (s - c[1]) / 1e3 if c else -1, (c[1] - c[0]) / 1e3 if c else -1))

"""Summarise a rocprofv3 --pmc CSV per kernel (mean over dispatches)."""
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for r in rows:
    k = r['Kernel_Name']
    agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    meta[k] = (r.get('VGPR_Count'), r.get('LDS_Block_Size'), r.get('Grid_Size'), r.get('Workgroup_Size'))
filt = sys.argv[2] if len(sys.argv) > 2 else "tcnn_amd"
for k, d in agg.items():
    if filt not in k:
        continue
    print(k[:110], "vgpr/lds/grid/wg", meta[k])
    print("   ", {c: f"{sum(v)/len(v):.4g}" for c, v in sorted(d.items())})

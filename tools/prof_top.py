"""Print the top kernels of a rocprofv3 --stats CSV summary (kernel_stats.csv) found under a directory."""
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
for path in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
    print(path)
    rows = list(csv.DictReader(open(path)))
    for r in rows[:12]:
        name = r["Name"]
        name = name if len(name) < 90 else name[:87] + "..."
        print(f'{float(r["AverageNs"]) / 1000:9.2f} us  x{r["Calls"]:>5}  {float(r["Percentage"]):6.2f}%  {name}')

"""Average PMC counters per dispatch from tools/archive/gpu_counters.sh output."""
import collections
import csv
import glob
import sys

res = collections.OrderedDict()
for f in sorted(glob.glob(sys.argv[1] + '/p*/run_counter_collection.csv')):
    agg = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        agg[r['Counter_Name']] += float(r['Counter_Value'])
        disp.add(r['Dispatch_Id'])
    for k, v in agg.items():
        res[k] = v / max(1, len(disp))
for k, v in res.items():
    print("%-32s %.4g" % (k, v))

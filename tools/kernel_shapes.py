# Kernel durations from a rocprofv3 kernel trace, grouped by (kernel, grid blocks): tools/kernel_shapes.py TRACE.csv
import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
by=collections.defaultdict(list)
for r in rows:
    k=r['Kernel_Name'].split('(')[0][-30:]
    g=int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])
    by[(k, g)].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in sorted(by.items()):
    v.sort(); print(k, len(v), 'median us %.1f min %.1f max %.1f' % (v[len(v)//2], v[0], v[-1]))

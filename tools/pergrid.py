"""Per-(kernel, grid) median / min duration of the wgrad and reduce launches from a rocprofv3 kernel trace."""
import csv,sys,collections
d=collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Kernel_Name']
    if 'wgrad' not in n and 'reduce' not in n: continue
    g=int(r.get('Grid_Size') or r.get('Grid_Size_X'))
    d[(n[:45],g)].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in sorted(d.items()):
    v=sorted(v); print(f"{k[0]:45s} grid={k[1]:8d} n={len(v):4d} median={v[len(v)//2]:8.1f} min={v[0]:8.1f}")

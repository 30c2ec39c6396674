import csv, glob, collections, sys
for v in sys.argv[1:]:
    tot = collections.defaultdict(float); disp = set()
    for f in sorted(glob.glob(f'{v}/p*/p_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            if 'tscan' not in r['Kernel_Name']: continue
            tot[r['Counter_Name']] += float(r['Counter_Value'])
            if f.endswith('p1/p_counter_collection.csv'): disp.add(r['Dispatch_Id'])
    nd = max(len(disp), 1)
    print(v, 'dispatches', nd)
    for k in sorted(tot): print(f'  {k:24s} {tot[k]/nd:.4g}')

"""Per-kernel average of PMC counters from rocprofv3 sqlite output dirs.
usage: pmc_db.py <dir> [<dir> ...] [--kernel REGEX]"""
import glob, re, sqlite3, sys, collections
args = [a for a in sys.argv[1:] if not a.startswith('--')]
rx = re.compile(sys.argv[sys.argv.index('--kernel') + 1]) if '--kernel' in sys.argv else None
if rx: args = [a for a in args if a != rx.pattern]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
    for f in glob.glob(d + '/**/*.db', recursive=True):
        db = sqlite3.connect(f)
        cols = [r[1] for r in db.execute("pragma table_info(counters_collection)")]
        for row in db.execute("select * from counters_collection"):
            r = dict(zip(cols, row))
            k = r.get('kernel_name', '').split('(')[0]
            if rx and not rx.search(k): continue
            agg[k][r['counter_name']].append(float(r['value']))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.4g}   (n={len(v)})")

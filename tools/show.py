"""print the bench JSON lines / bin_prof lines of gpurun_out logs"""
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            r = d.get('result', {})
            print(f, round(d['value'] / 1e9, 3), 'G/s', d['ms_per_step'], 'ms', d['phases_ms'], r.get('engine'), r.get('bins'))
        elif 'bin_prof' in l or 'Error' in l or 'error' in l:
            print(f, l.rstrip()[:400])

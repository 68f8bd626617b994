import json, sys, os
for f in sys.argv[1:]:
    if not os.path.exists(f) or not os.path.getsize(f):
        print(f, 'missing'); continue
    d = json.load(open(f))
    r = d['roofline']
    print(os.path.basename(f), d['ms_per_step'], round(d['value'] / 1e9, 2), 'cold', d['input']['cold_first_step_ms'],
          r['kernel'][:12], r['kernel_ms'], r['frac'], {k: v for k, v in d['phases_ms'].items()}, d['result']['bins'])
    print('   paths', d.get('paths'))
    if 'capacity' in d:
        c = d['capacity']
        print('   capacity', c['ms_per_step'], round(c['value'] / 1e9, 2), c['roofline']['kernel_ms'], c['roofline']['frac'], c['digest_ok'], c['cold_first_step_ms'], c['paths'])
    if 'host_input' in d:
        print('   host_input', d['host_input'])

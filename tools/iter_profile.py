"""Per-iteration breakdown of a wavefront frame from a rocprofv3 kernel trace."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_wf' in r['Kernel_Name']]
it, cur = [], {}
for r in rows:
    n = r['Kernel_Name']
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    targs = n.split('k_wf_trace<')[1].split('>')[0].split(', ') if 'k_wf_trace<' in n else None
    if targs and targs[2] == 'true':
        break  # the instrumented run follows
    if targs and targs[1] == 'false':
        cur = {'e': d, 't0': int(r['Start_Timestamp'])}
    elif 'k_wf_shade' in n:
        cur['sh'] = d
    elif targs:
        cur['s'] = d
    elif 'k_wf_advance' in n and 'e' in cur:
        cur['t1'] = int(r['End_Timestamp'])
        it.append(cur)
        cur = {}
print('iterations', len(it))
tot = lambda a, b: sum(x['e'] + x.get('sh', 0) + x.get('s', 0) for x in it[a:b]) / 1e3
print('frame span ms %.1f busy ms %.1f' % ((it[-1]['t1'] - it[0]['t0']) / 1e6, tot(0, len(it))))
step = 100
for a in range(0, len(it), step):
    b = min(len(it), a + step)
    print(f'iters {a:4d}-{b:4d}: {tot(a, b):7.1f} ms  extend avg {sum(x["e"] for x in it[a:b]) / (b - a):6.0f} us'
          f'  shadow avg {sum(x.get("s", 0) for x in it[a:b]) / (b - a):6.0f} us  shade avg '
          f'{sum(x.get("sh", 0) for x in it[a:b]) / (b - a):5.0f} us  min ext {min(x["e"] for x in it[a:b]):5.0f}')

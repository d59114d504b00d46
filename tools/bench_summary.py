import json,sys
for f in sys.argv[1:]:
    try:
        d=json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_us'])
    except Exception as e:
        print(f, 'ERR', e)

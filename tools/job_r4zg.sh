set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4zg; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac']);print({k:v for k,v in d.items() if 'lat' in k})" | cut -c1-1500

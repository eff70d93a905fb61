# bench.py option matrix on one GPU: each line must run and print its JSON
set -o pipefail
i=0
while read -r args; do
  i=$((i+1))
  timeout -k 10 200 python bench.py $args --steps 40 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/m$i.json 2> gpurun_out/m$i.err || { echo "FAIL: $args"; tail -5 gpurun_out/m$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/m$i.json').read().strip().splitlines()[-1]);print('$args |',round(d['value']/1e6,2),d['ms_per_step'],d['launch'],d['roofline']['kernel'],d['roofline']['frac'])"
done <<'LIST'
--wrapper neurips23_start_kit
--wrapper yaofeng --obs native
--no-graph
--config C5 --obs flat
--config C3 --batches 1
--config C2 --no-graph
--config C4 --obs native --batches 4
LIST

# Same-box A/B of library variants on one bench command: bash tools/debug/ab_lib.sh "<bench args>" lib1 lib2 ...
# (lib = nmmo_amd/lib/libnmmo_hip<suffix>.so; "base" = the default library); two alternating rounds.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ab && set -o pipefail
ARGS=$1; shift
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=nmmo_amd/lib/libnmmo_hip.so; else L=nmmo_amd/lib/libnmmo_hip_$v.so; fi
    NMMO_LIB=$L NMMO_ALLOW_STALE=1 timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline --no-extras \
      > gpurun_out/ab/${v}_$round.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/${v}_$round.json')); print('$v', $round, round(d['value']/1e6,2), d['kernel_ms'])"
  done
done

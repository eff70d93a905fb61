# Tick-kernel HBM request mix (why 2*FETCH_SIZE + WRITE_SIZE exceeds the algorithmic bytes):
# the TCC fabric read/write request counters by size class, one --pmc pass each, C2 and C3.
# FETCH_SIZE's x2 gfx950 correction holds only for wide 16-B/lane streaming reads
# (MI355X_MICROARCH.md §HBM); the size classes say how much of the tick's reads are narrow.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_reqs
mkdir -p $OUT
for c in C2 C3; do
  mkdir -p $OUT/$c
  for set in "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B" "TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"; do
    tag=$(echo $set | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/$c/$tag -o run -- \
      python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-extras > /dev/null 2> $OUT/$c/$tag.err || exit 1
  done
done

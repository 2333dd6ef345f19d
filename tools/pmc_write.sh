set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcw
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o run -- python $GRAFT_REPO_ROOT/tools/kprobe.py lin64 > $OUT/p$i.log 2>&1
done

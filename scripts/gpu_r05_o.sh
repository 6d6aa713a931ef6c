# Kernel traces of the Syn-10M bench line, bf16 and fp8 (adam_catchup 163 vs 428 us/step):
# which kernels run beside the catch-up launch in each precision.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for P in bf16 fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$P -o run -- python3 $R/bench.py \
    --precision $P --steps 40 --warmup 10 --no-cpu-baseline --probe-steps 20 > $O/$P.log 2>&1
  tail -1 $O/$P.log
done

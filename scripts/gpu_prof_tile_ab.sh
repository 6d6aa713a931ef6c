# rocprofv3 kernel stats of the Syn-1M fp8 bench with the old (64) and new (512) 64x64-tile thresholds of the fp32 GEMM.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/t3
cd /tmp && export TMPDIR=/tmp
export HVAE_GEMM_TILE64_MIN=64
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/t3/p64 -o run -- python3 $R/bench.py --workload syn1m --precision fp8 --steps 40 --warmup 3 --no-cpu-baseline --probe-steps 2 > $R/gpurun_out/t3/p64.log 2>&1
export HVAE_GEMM_TILE64_MIN=512
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/t3/p512 -o run -- python3 $R/bench.py --workload syn1m --precision fp8 --steps 40 --warmup 3 --no-cpu-baseline --probe-steps 2 > $R/gpurun_out/t3/p512.log 2>&1

# Kernel trace of the All_Beauty bench (graph-mode step timeline) and per-shape GEMM timings at B = 64 / 4096.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_traceab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload all_beauty --steps 400 --warmup 40 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
timeout -k 10 200 python3 $R/scripts/bench_gemm.py --batch 64 > $O/gemm_b64.jsonl 2> $O/gemm_b64.err
timeout -k 10 200 python3 $R/scripts/bench_gemm.py --batch 4096 > $O/gemm_b4096.jsonl 2> $O/gemm_b4096.err
timeout -k 10 200 python3 $R/scripts/bench_gemm.py --batch 4096 --d 768 > $O/gemm_b4096_d768.jsonl 2> $O/gemm_b4096_d768.err

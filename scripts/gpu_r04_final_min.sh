# Round-4 final evidence, compact (one call): every GPU test, smoke, the default bench (Syn-10M shard, bf16, CPU
# baseline), rocprofv3 kernel-trace stats of the default bench, the FETCH_SIZE / WRITE_SIZE passes of the default
# bench (stamped locally by scripts/pmc_to_traffic.py), and the other bench lines.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_final}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_syn10m.json 2> $O/bench_syn10m.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof.log 2>&1
KRX='k_dec|k_gemm|k_adam_lazy|k_encoder_sparse_fwd|k_mlp'
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_syn10m_fetch -o run -- python3 $R/bench.py --steps 8 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/pmc_syn10m_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_syn10m_write -o run -- python3 $R/bench.py --steps 8 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/pmc_syn10m_write.log 2>&1
cd $R
timeout -k 10 200 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 200 python -u bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
timeout -k 10 200 python -u bench.py --precision fp8 --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/bench_syn10m_fp8.json 2> $O/bench_syn10m_fp8.log

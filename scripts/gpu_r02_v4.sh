# Round-2 pass after decoder v4 + fused top-K: the default bench (Syn-10M shard, bf16, with the CPU baseline), its rocprofv3
# kernel-trace stats, FETCH/WRITE PMC passes of the same command, then every GPU test.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02v4
mkdir -p $O
timeout -k 10 420 python -u bench.py --steps 30 --warmup 5 --probe-steps 5 > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
BEN="python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --probe-steps 3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $BEN > $O/prof.log 2>&1
KRX='k_dec4_bf16|k_dec_finalize|k_gemm|k_adam_lazy|k_encoder'
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_fetch -o run -- $BEN > $O/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_write -o run -- $BEN > $O/pmc_write.log 2>&1
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1

# Version 4 with GEMM1's conflict-free row map (default build) against the natural row order
# (build_var/libhvae_oldmap.so, DEC4_ROWMAP=0x3210): d = 768 parity tests on the default, the sweep at the
# Syn-10M shard in alternating processes, then LDS / MFMA counters of the default.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rowmap
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_train.py -m gpu -x -q -k "768 or versions or fused_step or d768" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/new_$i.jsonl 2>&1
  HVAE_LIB=$R/build_var/libhvae_oldmap.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/old_$i.jsonl 2>&1
done
cd /tmp && export TMPDIR=/tmp
DEC="python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec4_bf16' --output-format csv -d $O/p1 -o run -- $DEC > $O/p1.log 2>&1
python3 $R/scripts/pmc_summary.py $O/p1 > $O/pmc_summary.txt

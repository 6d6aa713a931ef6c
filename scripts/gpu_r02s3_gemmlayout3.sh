# GEMM fast-path stage image, layout 1 (default build: chunk stride R, rows XOR-swizzled in their chunk)
# against layout 0 (build_var/libhvae_gemmold.so): parity on the default, per-shape timing at B = 4096, d = 384
# and 768, alternating processes, then LDS counters of the default.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemmlayout3
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gemm or pair" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
  for d in 384 768; do
    timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $d --reps 50 --no-torch > $O/new_d${d}_$i.txt 2>&1
    HVAE_LIB=$R/build_var/libhvae_gemmold.so timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $d --reps 50 --no-torch > $O/old_d${d}_$i.txt 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex 'k_gemm' --output-format csv -d $O/pmc -o run -- python3 $R/bench.py --workload syn1m --steps 5 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/pmc.log 2>&1
python3 $R/scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt

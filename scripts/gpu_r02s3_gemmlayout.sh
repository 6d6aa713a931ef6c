# GEMM fast path with the conflict-free stage image (default build, FAST_LAYOUT=1) against the first layout
# (build_var/libhvae_gemmold.so): GEMM / pair parity tests on the default, per-shape timing at B = 4096 for
# d = 384 and 768 in alternating processes, then the Syn-1M and Syn-10M steps on each, and LDS counters.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemmlayout
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gemm or pair" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
  for d in 384 768; do
    timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $d --reps 50 --no-torch > $O/new_d${d}_$i.txt 2>&1
    HVAE_LIB=$R/build_var/libhvae_gemmold.so timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $d --reps 50 --no-torch > $O/old_d${d}_$i.txt 2>&1
  done
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/new_s1m_$i.json 2> $O/new_s1m_$i.log
  HVAE_LIB=$R/build_var/libhvae_gemmold.so timeout -k 10 200 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/old_s1m_$i.json 2> $O/old_s1m_$i.log
done
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/new_s10m.json 2> $O/new_s10m.log
HVAE_LIB=$R/build_var/libhvae_gemmold.so timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/old_s10m.json 2> $O/old_s10m.log
cd /tmp && export TMPDIR=/tmp
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex 'k_gemm' --output-format csv -d $O/pmc -o run -- python3 $R/bench.py --workload syn1m --steps 5 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/pmc.log 2>&1
python3 $R/scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt

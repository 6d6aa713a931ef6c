# Round 6, call A: (1) the LDS-DMA issue-form probe (scripts/probe_dma_issue.hip); (2) the version-5 sweep's per-tile
# phase budget from timing builds (with and without its DMA) and the global_load_lds arm's budget; (3) the sweep's
# wall time, product vs global_load_lds, alternating processes; (4) the d = 768 decoder parity tests on the
# global_load_lds build; (5) where the step joins the row-gradient plan (HVAE_PLAN_JOIN apply | fwd) at Syn-10M
# and Syn-1M, alternating; (6) the GPU tests this round's ADVICE fixes touch.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
timeout -k 10 120 build_probe/probe_dma_issue 2000 1 > $O/dma_issue_reads.jsonl 2> $O/dma_issue.err || exit 1
timeout -k 10 120 build_probe/probe_dma_issue 2000 0 > $O/dma_issue_noreads.jsonl 2>> $O/dma_issue.err || exit 1
for v in d5tm d5tm_nodma d5glds_tm; do
  HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 150 python -u scripts/probe_dec5_phases.py --label $v \
    >> $O/dec5_phases.jsonl 2>> $O/dec5_phases.err || exit 1
done
for r in 1 2 3; do
  for v in prod d5glds; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 150 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 8 \
      2>> $O/dec_ab.err | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" >> $O/dec_ab.jsonl || exit 1
  done
done
HVAE_LIB=build_var/libhvae_d5glds.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large_step.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -k "768 or syn10m" > $O/pytest_glds.log 2>&1 || exit 1
for r in 1 2; do
  for j in apply fwd; do
    for wl in syn10m syn1m; do
      HVAE_PLAN_JOIN=$j timeout -k 10 300 python -u bench.py --workload $wl --steps 100 --warmup 20 --no-cpu-baseline \
        --probe-steps 3 2>> $O/join.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'join':'$j','workload':'$wl','ms':d['ms_per_step'],'value':d['value']}))" >> $O/join_ab.jsonl || exit 1
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dp.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "gemm or dp" > $O/pytest_advice.log 2>&1 || exit 1
echo done > $O/done

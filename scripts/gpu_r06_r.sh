# Round 6, call R: the two-users-per-block finalize (k_dec_finalize_pair): bitwise against the one-user kernel and
# the decoder / train-step tests, then bench A/B (HVAE_FIN_PAIR=0/1) at Syn-1M and All_Beauty (the Syn-10M finalize
# at d = 768 keeps one user per block); and the CSR catch-up unroll A/B in the A/B library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "decoder or finalize or step or golden" > $O/pytest_pair.log 2>&1 || exit 1
ab() {  # pair workload precision
  HVAE_FIN_PAIR=$1 timeout -k 10 300 python -u bench.py --workload $2 --precision $3 --steps 200 --warmup 30 \
    --no-cpu-baseline --probe-steps 3 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'fin_pair':$1,'workload':'$2','precision':'$3','ms':d['ms_per_step'],'finalize_us':d['launch_us']['decoder_finalize']['avg_us']}))" >> $O/pair_ab.jsonl || exit 2
}
for r in 1 2; do
  for p in 0 1; do ab $p syn1m bf16; done
  for p in 0 1; do ab $p all_beauty bf16; done
done
bash scripts/gpu_r06_q.sh || exit 3
echo done > $O/done

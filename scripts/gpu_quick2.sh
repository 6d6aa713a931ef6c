set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
timeout -k 10 120 python scripts/bench_decoder.py --nb 64 --N 12101 --D 384 --reps 50 --train --probe decoder_finalize 2>&1 | grep -v amdgpu.ids > gpurun_out/dec_fin.log
timeout -k 10 120 python scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --reps 10 --train --probe decoder_finalize 2>&1 | grep -v amdgpu.ids >> gpurun_out/dec_fin.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
timeout -k 10 400 python bench.py --workload syn1m --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/bench_syn1m.log 2>&1

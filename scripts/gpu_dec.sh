# Decoder: parity tests of the sweep, then timing on the bench shapes.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "decoder" --timeout 120 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1
B=scripts/bench_decoder.py
run() { echo "# $1 $2" >> gpurun_out/dec_ab.log; env $1 timeout -k 10 120 python $B $2 --reps 20 2>&1 | grep -v amdgpu.ids >> gpurun_out/dec_ab.log; }
S1="--nb 4096 --N 100000 --D 384"
run "X=1" "$S1"
run "HVAE_DEC_DS=2 HVAE_DEC_NW=8" "$S1"
run "X=1" "--nb 64 --N 12101 --D 384"
run "X=1" "--nb 4096 --N 200000 --D 768"

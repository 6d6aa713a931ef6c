# Stamp the round-6 final PMC passes (scripts/gpu_r06_final_a.sh) into profiles/ (run in the build container after
# the call's gpurun_out/ merged back).
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/${OUT:-r06_final}
python3 scripts/pmc_to_traffic.py syn10m $O/pmc_syn10m_fetch $O/pmc_syn10m_write k_dec5_bf16=decoder_sweep k_dec_finalize=decoder_finalize k_gemm=gemm k_adam_lazy=adam_rows k_encoder_sparse_fwd=encoder_fwd > /dev/null
python3 scripts/pmc_to_traffic.py syn10m_fp8 $O/pmc_syn10m_fp8_fetch $O/pmc_syn10m_fp8_write k_dec5_f8=decoder_sweep k_dec_finalize=decoder_finalize k_gemm=gemm k_adam_lazy=adam_rows k_encoder_sparse_fwd=encoder_fwd > /dev/null
python3 scripts/pmc_to_traffic.py syn1m $O/pmc_syn1m_fetch $O/pmc_syn1m_write k_dec2_bf16=decoder_sweep k_dec_finalize=decoder_finalize k_gemm=gemm k_adam_lazy=adam_rows k_encoder_sparse_fwd=encoder_fwd > /dev/null
python3 scripts/pmc_to_traffic.py syn1m_fp8 $O/pmc_syn1m_fp8_fetch $O/pmc_syn1m_fp8_write k_dec_fp8=decoder_sweep k_dec_finalize=decoder_finalize k_gemm=gemm k_adam_lazy=adam_rows k_encoder_sparse_fwd=encoder_fwd > /dev/null
python3 scripts/pmc_to_traffic.py all_beauty $O/pmc_all_beauty_fetch $O/pmc_all_beauty_write k_dec2_bf16=decoder_sweep k_dec_finalize=decoder_finalize k_gemm=gemm k_adam_lazy=adam_rows k_mlp_fwd=mlp_fwd k_mlp_bwd=mlp_bwd > /dev/null
python3 scripts/pmc_sq_stamp.py profiles/pmc_sq_dec5_syn10m.json bf16=$O/sq_bf16 fp8=$O/sq_fp8
python3 -c "
import json
for w in ['syn10m','syn10m_fp8','syn1m','syn1m_fp8','all_beauty']:
    d=json.load(open(f'profiles/pmc_{w}.json')); print(w, d['src_sha'], {k: v['hbm_bytes_per_launch'] for k, v in d.items() if isinstance(v, dict)})
"

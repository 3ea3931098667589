set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_f0.so timeout -k 10 200 python scripts/check_bitwise.py gpurun_out/bw_f0.npz && ADMM_TOMO_LIB=variants/lib_f1.so timeout -k 10 200 python scripts/check_bitwise.py gpurun_out/bw_f1.npz && python scripts/check_bitwise.py --compare gpurun_out/bw_f0.npz gpurun_out/bw_f1.npz

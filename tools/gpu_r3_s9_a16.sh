export TMPDIR=/tmp
CZ_LIB=$PWD/jeromq_amd/libcz_a16s.so timeout -k 10 400 python -u -m pytest tests/test_gpu_layouts_full.py tests/test_gpu_segments.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_a16s.log 2>&1 || { tail -30 gpurun_out/pytest_a16s.log; exit 3; }
tail -1 gpurun_out/pytest_a16s.log
CONFIGS="--config zipf --in-align 8 --out-align 8;--config zipf --out-align 1;--config zipf --out-align 16;--config zipf" bash tools/gpu_ab_all.sh libcz_rel.so libcz_a16.so libcz_a16s.so

cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== full gpu suite, product library"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s4_pytest.log 2>&1 || { tail -30 gpurun_out/r4s4_pytest.log; exit 2; }
tail -1 gpurun_out/r4s4_pytest.log
echo "== flush2 parity (seal paths)"
CZ_LIB=$PWD/jeromq_amd/libcz_flush2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_box.py tests/test_gpu_layouts_full.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s4_pytest_flush2.log 2>&1 || { tail -30 gpurun_out/r4s4_pytest_flush2.log; exit 3; }
tail -1 gpurun_out/r4s4_pytest_flush2.log
echo "== ab_lib r4 / flush2 / w2"
timeout -k 10 600 python tools/ab_lib.py jeromq_amd/libcz_r4.so jeromq_amd/libcz_flush2.so jeromq_amd/libcz_w2.so --spec 4k --spec 4k_box --rounds 8 > gpurun_out/r4s4_ab.log 2>&1 || { tail gpurun_out/r4s4_ab.log; exit 4; }
grep -v amdgpu.ids gpurun_out/r4s4_ab.log
echo "== ab_cfg seal/open, product"
timeout -k 10 400 python tools/ab_cfg.py 4k open4k 4k open4k "open4k --plain-stride 4224" 4k_box --rounds 8 > gpurun_out/r4s4_ab_cfg.log 2>&1 || { tail gpurun_out/r4s4_ab_cfg.log; exit 5; }
grep -v amdgpu.ids gpurun_out/r4s4_ab_cfg.log
echo "== clocks"
timeout -k 10 500 bash tools/gpu_clock_ab.sh libcz_r4.so libcz_flush2.so || exit 6
CZ_CLOCK_CONFIG=open4k timeout -k 10 300 bash tools/gpu_clock_ab.sh libcz_r4.so || exit 7

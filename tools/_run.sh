cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== full gpu suite with carry lib"
CZ_LIB=$PWD/jeromq_amd/libcz_carry.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s3_pytest_carry.log 2>&1 || { tail -30 gpurun_out/r4s3_pytest_carry.log; exit 2; }
tail -1 gpurun_out/r4s3_pytest_carry.log
echo "== ab_lib"
timeout -k 10 900 python tools/ab_lib.py jeromq_amd/libcz_base.so jeromq_amd/libcz_tail2.so jeromq_amd/libcz_fence.so jeromq_amd/libcz_w2.so jeromq_amd/libcz_al8x4.so jeromq_amd/libcz_carry.so jeromq_amd/libcz_carry3.so --spec 100b --spec 4k --spec 4k_box --spec open4k --spec "open4k --out-stride 4129" --spec "open4k --out-stride 4136" --spec "open4k --out-stride 133 --in-stride 112" --spec 4k_dense --spec zipf --spec "zipf_open --in-align 8 --out-align 8" --rounds 5 > gpurun_out/r4s3_ab.log 2>&1 || { tail gpurun_out/r4s3_ab.log; exit 3; }
cat gpurun_out/r4s3_ab.log | grep -v amdgpu.ids
echo "== ab_cfg strides"
CZ_LIB=$PWD/jeromq_amd/libcz_fence.so timeout -k 10 400 python tools/ab_cfg.py 4k open4k "open4k --plain-stride 4224" "open4k --plain-stride 4352" 4k_box --rounds 8 > gpurun_out/r4s3_ab_cfg.log 2>&1 || { tail gpurun_out/r4s3_ab_cfg.log; exit 4; }
cat gpurun_out/r4s3_ab_cfg.log | grep -v amdgpu.ids

cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== full gpu suite with fence lib"
CZ_LIB=$PWD/jeromq_amd/libcz_fence.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s3_pytest_fence.log 2>&1 || { tail -30 gpurun_out/r4s3_pytest_fence.log; exit 2; }
tail -1 gpurun_out/r4s3_pytest_fence.log
echo "== ab_lib base/tail2/fence"
timeout -k 10 900 python tools/ab_lib.py jeromq_amd/libcz_base.so jeromq_amd/libcz_tail2.so jeromq_amd/libcz_fence.so --spec 100b --spec 4k --spec 4k_box --spec open4k --spec "open4k --out-stride 4129" --spec "open4k --out-stride 133 --in-stride 112" --spec 4k_dense --spec zipf --spec "zipf_open --in-align 8 --out-align 8" --rounds 6 > gpurun_out/r4s3_ab.log 2>&1 || { tail gpurun_out/r4s3_ab.log; exit 3; }
cat gpurun_out/r4s3_ab.log | grep -v amdgpu.ids

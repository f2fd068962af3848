cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u tools/ab_lib.py --rounds 12 --steps 5 --spec 4k --spec 4k_box --spec 100b jeromq_amd/libcz_base.so jeromq_amd/libcz_hold.so jeromq_amd/libcz_base.so jeromq_amd/libcz_hold.so > gpurun_out/r5_ab_hold.log 2>&1 && \
bash tools/gpu_clock_ab.sh libcz_base.so libcz_hold.so libcz_base.so libcz_hold.so > gpurun_out/r5_clock_hold.log 2>&1

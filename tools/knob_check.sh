# occupancy / segment-length re-check of the final kernel (bench.py per variant, interleaved)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=fast_kinematic_simulator_amd/libfks_hip.so
W6=build/variants/libfks_w6.so
timeout -k 10 1100 python tools/variant_bench.py $L $W6 $L+segment-steps=10 $L+segment-steps=18 $L $W6 $L+segment-steps=10 $L+segment-steps=18 > gpurun_out/r03q_knobs.log 2>&1 || exit 1
echo done

# default kernel vs the joint-space proof, interleaved (cfg3 bench.py lines)
export TMPDIR=/tmp
L=fast_kinematic_simulator_amd/libfks_hip.so
timeout -k 10 800 python tools/variant_bench.py $L $L+joint-proof $L $L+joint-proof $L $L+joint-proof 2>&1 | cut -c1-140

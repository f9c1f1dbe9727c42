# scheduling A/B (contact-carry thresholds) + bench.py through torchrun (world 1, RCCL)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=fast_kinematic_simulator_amd/libfks_hip.so
timeout -k 10 900 python tools/variant_bench.py $NEW build/variants/libfks_h1.so build/variants/libfks_h7.so $NEW build/variants/libfks_h1.so build/variants/libfks_h7.so > gpurun_out/r03n_sched_ab.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03n_torchrun_w1.json 2> gpurun_out/r03n_torchrun_w1.err || exit 1
echo done

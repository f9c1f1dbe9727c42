# round-end evidence for the committed build, then an A/B of one candidate variant on cfg3/cfg4
# usage: bash tools/final_and_ab.sh <tag> <candidate.so>
TAG=$1; C=$2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/final_round.sh $TAG || exit $?
NEW=fast_kinematic_simulator_amd/libfks_hip.so
timeout -k 10 700 python tools/variant_bench.py $NEW $C $NEW $C $NEW $C > gpurun_out/${TAG}_cand_ab_cfg3.log 2>&1 || exit 1
timeout -k 10 600 python tools/variant_bench.py $NEW $C $NEW $C --workload cfg4 --no-config-check > gpurun_out/${TAG}_cand_ab_cfg4.log 2>&1 || exit 1
echo all_done

# A/B of the walk search's state/stateless threshold on the cfg3 bench; needs a build whose launch_nn_walk_search reads CLRRT_WALK_STATE_MAX (not the shipped one).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abw
for v in 1280 2560 1280 4096 2560; do
  CLRRT_WALK_STATE_MAX=$v timeout -k 10 120 python3 -u bench.py --no-cpu > gpurun_out/abw/s$v.$RANDOM.json 2>/dev/null
done
echo done

# Round 5: EXACT fix-up statistics (why a round's committed prefix ends) on cfg3.
set -e
tag=${1:-r05e}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 -u tools/exact_fixup_stats.py 2000 > $out/exact_fixup_stats.txt 2>&1

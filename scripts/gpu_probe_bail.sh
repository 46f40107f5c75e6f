set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== stats"; OGBX_LIB=$PWD/_abx/libogbx_stats.so timeout -k 10 200 python scripts/probe_bail.py || exit 3

set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in stats serstats; do echo "== $v"; OGBX_LIB=$PWD/_ab/libogbx_$v.so timeout -k 10 200 python scripts/probe_bail.py || exit 3; done

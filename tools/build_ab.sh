#!/bin/bash
# Build the kernel library of git revision REV (default HEAD) into
# chiaswarm_amd/lib/ab/libcsk_old.so for a same-box A/B against the working
# tree's libcsk.so (tools/gpu/lib_ab.sh, CSK_LIB_PATH).  CPU only.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/csk_ab_wt
rm -rf $WT
git -C $ROOT worktree prune
git -C $ROOT worktree add --detach $WT $REV > /dev/null
(cd $WT && python -m chiaswarm_amd._build > /dev/null)
mkdir -p $ROOT/chiaswarm_amd/lib/ab
cp $WT/chiaswarm_amd/lib/libcsk.so $ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
git -C $ROOT worktree remove --force $WT
echo "built $REV -> chiaswarm_amd/lib/ab/libcsk_old.so"

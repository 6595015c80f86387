#!/bin/bash
# Build a git revision's library AND its Python package into ab/<name>/ (ab/<name>/sr_amd +
# ab/<name>/lib/libsr_amd.so): A/B runs select it with SR_AMD_PKG=ab/<name> (older packages bind only
# the symbols of their own library).  usage: tools/ab_lib.sh <rev> <name> [EXTRA flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2; shift 2
wt=/tmp/ab_wt_$name
rm -rf "$wt"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f --detach "$wt" "$rev" > /dev/null
make -s -j8 -C "$wt/symbolicregression.jl_amd" EXTRA="$*"
rm -rf "$ROOT/ab/$name"; mkdir -p "$ROOT/ab/$name/lib"
cp "$wt/symbolicregression.jl_amd/lib/libsr_amd.so" "$ROOT/ab/$name/lib/libsr_amd.so"
cp -r "$wt/symbolicregression.jl_amd/sr_amd" "$ROOT/ab/$name/sr_amd"
git -C "$ROOT" worktree remove --force "$wt"
echo "built ab/$name from $rev"

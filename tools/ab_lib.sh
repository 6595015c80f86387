#!/bin/bash
# Build libsr_amd.so of a git revision into ab/<name>/libsr_amd.so (A/B runs select it with
# SR_AMD_LIB=ab/<name>/libsr_amd.so).  usage: tools/ab_lib.sh <rev> <name> [EXTRA flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2; shift 2
wt=/tmp/ab_wt_$name
rm -rf "$wt"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f --detach "$wt" "$rev" > /dev/null
make -s -j8 -C "$wt/symbolicregression.jl_amd" EXTRA="$*"
mkdir -p "$ROOT/ab/$name"
cp "$wt/symbolicregression.jl_amd/lib/libsr_amd.so" "$ROOT/ab/$name/libsr_amd.so"
git -C "$ROOT" worktree remove --force "$wt"
echo "built ab/$name/libsr_amd.so from $rev"

#!/bin/bash
# Build libmpo.so of other git revisions into ab_libs/<name>/libmpo.so for same-box
# A/B runs (a probe selects one with MPO_LIB_AB=ab_libs/<name>/libmpo.so, read by scripts/ab_lib.py).
#   scripts/ab_libs.sh name=rev [name=rev ...]
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD
for spec in "$@"; do
  name=${spec%%=*}; rev=${spec#*=}
  wt=/tmp/ab_wt_$name
  rm -rf "$wt"; git worktree prune
  git worktree add --detach "$wt" "$rev" > /dev/null
  make -C "$wt/mpi_opt_amd/csrc" -j8 > /tmp/ab_build_$name.log 2>&1
  mkdir -p "ab_libs/$name"
  cp "$wt/mpi_opt_amd/libmpo.so" "ab_libs/$name/libmpo.so"
  git worktree remove --force "$wt"
  echo "ab_libs/$name/libmpo.so <- $rev"
done

#!/bin/bash
# Builds the codec library of a git revision (default HEAD) into abl/<name>.so for scripts/ab_rows.py
# (A/B of a working-tree change against the committed kernel).  Usage: scripts/ab_git.sh name [rev] [-Dflags...]
set -e
cd "$(dirname "$0")/.."
name=$1; rev=${2:-HEAD}; shift; shift || true
d=abl/src_$name
rm -rf $d && mkdir -p $d/pkg/csrc $d/include
for f in sbe_codec.hip seqnum.hpp order_json.hpp; do git show $rev:aeron-cluster-client-cpp_amd/csrc/$f > $d/pkg/csrc/$f; done
git show $rev:include/sbecodec.h > $d/include/sbecodec.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" $d/pkg/csrc/sbe_codec.hip -o abl/$name.so -ldl
echo built abl/$name.so from $rev

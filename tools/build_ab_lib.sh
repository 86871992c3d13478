#!/bin/bash
# Build libscgib.so from a git revision (default HEAD) into s-cgib_amd/libscgib_ab.so,
# for A/B runs against the working tree: SCGIB_LIB=$PWD/s-cgib_amd/libscgib_ab.so
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" s-cgib_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/s-cgib_amd/csrc" >/dev/null
cp "$tmp/s-cgib_amd/libscgib.so" "$root/s-cgib_amd/libscgib_ab.so"
rm -rf "$tmp"
echo "built $rev -> s-cgib_amd/libscgib_ab.so"

#!/bin/bash
# Build libscgib.so from a git revision (default HEAD) into s-cgib_amd/libscgib_ab.so,
# for A/B runs against the working tree: SCGIB_LIB=$PWD/s-cgib_amd/libscgib_ab.so
# (EXTRA="-DKNOB=..." passes extra compiler flags; rev "WORKTREE" = current files)
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
if [ "$rev" = WORKTREE ]; then
  mkdir -p "$tmp/s-cgib_amd" && cp -r "$root/s-cgib_amd/csrc" "$tmp/s-cgib_amd/" && cp -r "$root/include" "$tmp/"
else
  git -C "$root" archive "$rev" s-cgib_amd/csrc include | tar -x -C "$tmp"
fi
make -s -j8 -C "$tmp/s-cgib_amd/csrc" EXTRA="${EXTRA:-}" >/dev/null
cp "$tmp/s-cgib_amd/libscgib.so" "$root/s-cgib_amd/${OUT:-libscgib_ab.so}"
rm -rf "$tmp"
echo "built $rev -> s-cgib_amd/${OUT:-libscgib_ab.so}"

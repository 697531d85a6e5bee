# Build build/var/libgqmap_base.so from the committed tree (HEAD) and
# build/var/libgqmap_new.so from the working tree, for scripts/ab_kernel.sh.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/gq_base && git -C "$ROOT" worktree remove --force /tmp/gq_base 2>/dev/null || true
git -C "$ROOT" worktree add -f /tmp/gq_base HEAD -q
make -s -j8 -C /tmp/gq_base/gqmap-opticalflow_amd >/dev/null
mkdir -p "$ROOT/gqmap-opticalflow_amd/build/var"
rm -f "$ROOT"/gqmap-opticalflow_amd/build/var/libgqmap_*.so
cp /tmp/gq_base/gqmap-opticalflow_amd/libgqmap.so "$ROOT/gqmap-opticalflow_amd/build/var/libgqmap_base.so"
make -s -j8 -C "$ROOT/gqmap-opticalflow_amd" >/dev/null
cp "$ROOT/gqmap-opticalflow_amd/libgqmap.so" "$ROOT/gqmap-opticalflow_amd/build/var/libgqmap_new.so"
git -C "$ROOT" worktree remove --force /tmp/gq_base
ls "$ROOT/gqmap-opticalflow_amd/build/var/"

# lib/ab/libx2g_base.so = libx2g.so built from a git revision (default HEAD), for step A/B runs
# against the working tree's build (scripts/ab_run.sh, scripts/ab_prof.sh)
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/x2g_base.XXXXXX)
git -C "$ROOT" worktree add --detach "$WT" "$REV" >/dev/null
make -C "$WT/x2-gnn_amd" -j8 >/dev/null
mkdir -p "$ROOT/x2-gnn_amd/lib/ab"
cp "$WT/x2-gnn_amd/lib/libx2g.so" "$ROOT/x2-gnn_amd/lib/ab/libx2g_base.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "base = $(git -C "$ROOT" rev-parse --short "$REV")"

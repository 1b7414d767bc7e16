#!/bin/bash
# ab_base/ = the files bench.py --step-only needs (bench.py, the x2gnn package, its built libx2g.so, the
# oracle package, the profile summaries bench.py reads) as of a git revision (default HEAD), for step
# A/B runs of host-side (Python) changes: scripts/step_ab.py runs a variant's bench.py from the
# directory its AB_ROOT names.  ab_base/ is git-ignored and travels to the GPU box with the tree.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/x2g_base.XXXXXX)
git -C "$ROOT" worktree add --detach "$WT" "$REV" >/dev/null
make -C "$WT/x2-gnn_amd" -j8 >/dev/null
rm -rf "$ROOT/ab_base"
mkdir -p "$ROOT/ab_base/x2-gnn_amd/lib" "$ROOT/ab_base/profiles"
cp "$WT/bench.py" "$ROOT/ab_base/"
cp -r "$WT/x2-gnn_amd/x2gnn" "$ROOT/ab_base/x2-gnn_amd/"
cp "$WT/x2-gnn_amd/lib/libx2g.so" "$ROOT/ab_base/x2-gnn_amd/lib/"
cp -r "$WT/oracle" "$ROOT/ab_base/"
cp "$WT"/profiles/*.json "$ROOT/ab_base/profiles/"
mkdir -p "$ROOT/ab_base/tests/golden"
cp "$WT"/tests/golden/aid_geom.npz "$ROOT/ab_base/tests/golden/"  # config 5's geometries (bench --workload aid_infer)
git -C "$ROOT" worktree remove --force "$WT"
echo "ab_base = $(git -C "$ROOT" rev-parse --short "$REV")"

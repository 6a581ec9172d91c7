#!/bin/bash
# Build the A (git ref, default HEAD) and B (working tree) libraries for tools/ab_libs.sh.
set -eu
cd "$(dirname "$0")/.."
REF=${1:-HEAD}
mkdir -p gaussianrenderer_amd/lib/ab
make -s >/dev/null && cp gaussianrenderer_amd/lib/libgsr.so gaussianrenderer_amd/lib/ab/libgsr_B.so
T=$(mktemp -d); git worktree add -q --detach "$T" "$REF"
make -s -C "$T" gaussianrenderer_amd/lib/libgsr.so >/dev/null && cp "$T/gaussianrenderer_amd/lib/libgsr.so" gaussianrenderer_amd/lib/ab/libgsr_A.so
git worktree remove --force "$T"
ls -la gaussianrenderer_amd/lib/ab

#!/bin/bash
# Build A (working tree, EXTRA_A flags) and B (working tree, EXTRA_B flags) libraries for
# tools/ab_libs.sh: compile-time variants of the same source.
set -eu
cd "$(dirname "$0")/.."
mkdir -p gaussianrenderer_amd/lib/ab
for L in A B; do
  V=EXTRA_$L
  rm -f build/obj/gsr_kernels.o
  make -s EXTRA_HIPFLAGS="${!V:-}" gaussianrenderer_amd/lib/libgsr.so >/dev/null
  cp gaussianrenderer_amd/lib/libgsr.so gaussianrenderer_amd/lib/ab/libgsr_$L.so
done
rm -f build/obj/gsr_kernels.o
make -s gaussianrenderer_amd/lib/libgsr.so >/dev/null
ls -la gaussianrenderer_amd/lib/ab

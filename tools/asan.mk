# tools/asan.mk — host-code sanitizer build ("race detection /
# sanitizers"): AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code only.
#
#   build/asan/libgsr.so      libgsr.so with the host runtime, the PLY parser and the GL
#                             interop instrumented (the gfx950 kernels object is the
#                             normal one: device code is never sanitized here)
#   build/asan/liboracle.so   the C oracle, instrumented
#
# Both use clang's sanitizer runtime (ROCm's LLVM), so one preloaded runtime serves a
# Python process that loads both (tests/test_sanitizers.py).  Run through the top-level
# `make asan`.  CPU only; no GPU run loads these libraries.
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CLANG ?= $(ROCM)/lib/llvm/bin/clang
ARCH ?= gfx950
OUT = build/asan
SRC = gaussianrenderer_amd/csrc
# host-only compiles (-x c++): the sanitizer flags apply to host code only
SAN = -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
      -fno-sanitize-recover=all -fno-omit-frame-pointer -g
HOSTFLAGS = -O1 -std=c++17 -I$(ROCM)/include -ffp-contract=off -fno-fast-math -fPIC -Wall -Iinclude -I$(SRC) \
            -D__HIP_PLATFORM_AMD__
HDRS = include/gsr.h include/gsr_types.h include/gsr_detmath.h $(SRC)/gsr_internal.h

all: $(OUT)/libgsr.so $(OUT)/liboracle.so

$(OUT)/%.o: $(SRC)/%.cpp $(HDRS)
	mkdir -p $(OUT)
	$(HIPCC) $(HOSTFLAGS) $(SAN) -x c++ -c $< -o $@

$(OUT)/libgsr.so: build/obj/gsr_kernels.o $(OUT)/gsr_runtime.o $(OUT)/gsr_ply.o $(OUT)/gsr_gl.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	    -shared-libsan -o $@ $^ -ldl -Wl,-soname,libgsr.so

$(OUT)/liboracle.so: oracle/gsr_oracle.c oracle/gsr_oracle.h include/gsr_detmath.h include/gsr_types.h
	mkdir -p $(OUT)
	$(CLANG) -O1 -ffp-contract=off -fno-fast-math -std=gnu11 -fopenmp -fPIC -shared -Wall \
	    -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -shared-libsan \
	    -o $@ oracle/gsr_oracle.c -lm -Wl,-rpath,$(ROCM)/lib/llvm/lib

.PHONY: all

# Top-level build: the product library (gfx950 HIP + host runtime) and the
# test-only oracle.  `make` is what __graft_entry__.build() runs.
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8

# -ffp-contract=off: no implicit FMA anywhere (bit parity with the oracle);
# no fast-math: IEEE division/sqrt (HIP's default correctly rounded fp32 div/sqrt).
HIPFLAGS = $(EXTRA_HIPFLAGS) -O3 -std=c++17 --offload-arch=$(ARCH) -mcode-object-version=5 -ffp-contract=off -fno-fast-math -fPIC \
           -Wall -Wno-unused-result -Iinclude -Igaussianrenderer_amd/csrc
HOSTFLAGS = -O2 -std=c++17 -I$(ROCM)/include -ffp-contract=off -fno-fast-math -fPIC -Wall -Iinclude -Igaussianrenderer_amd/csrc

LIB = gaussianrenderer_amd/lib/libgsr.so
OBJDIR = build/obj
SRCDIR = gaussianrenderer_amd/csrc
HDRS = include/gsr.h include/gsr_types.h include/gsr_detmath.h $(SRCDIR)/gsr_internal.h

all: $(LIB) oracle

$(OBJDIR)/gsr_kernels.o: $(SRCDIR)/gsr_kernels.hip $(HDRS)
	mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/gsr_runtime.o: $(SRCDIR)/gsr_runtime.cpp $(HDRS)
	mkdir -p $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJDIR)/gsr_ply.o: $(SRCDIR)/gsr_ply.cpp $(HDRS)
	mkdir -p $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJDIR)/gsr_gl.o: $(SRCDIR)/gsr_gl.cpp $(HDRS) include/gsr_gl.h
	mkdir -p $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(LIB): $(OBJDIR)/gsr_kernels.o $(OBJDIR)/gsr_runtime.o $(OBJDIR)/gsr_ply.o $(OBJDIR)/gsr_gl.o
	mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -Wl,-soname,libgsr.so

oracle: $(LIB)
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# host-code ASan + UBSan build of libgsr.so and the oracle (tools/asan.mk; CPU tests only)
asan: $(OBJDIR)/gsr_kernels.o
	$(MAKE) -f tools/asan.mk -j $(JOBS)

.PHONY: asan

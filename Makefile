# Top-level build: the HIP engine (gfx950) + the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := pmdfc_amd/csrc
LIBDIR := pmdfc_amd/lib
LIB := $(LIBDIR)/libpmdfc_cceh.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
SRCS := $(CSRC)/cceh_kernels.hip $(CSRC)/bucket.hip $(CSRC)/bloom.hip $(CSRC)/cceh_engine.hip
HDRS := $(CSRC)/cceh_device.h $(CSRC)/cceh_kernels.h include/pmdfc_cceh.h
OBJS := $(patsubst $(CSRC)/%.hip,$(LIBDIR)/obj/%.o,$(SRCS))

all: $(LIB) oracle

$(LIBDIR)/obj/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C oracle liboracle.so

clean:
	rm -rf $(LIBDIR) oracle/liboracle.so

.PHONY: all oracle clean

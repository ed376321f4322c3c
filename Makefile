# Top-level build: the HIP engine (gfx950) + the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := pmdfc_amd/csrc
LIBDIR := pmdfc_amd/lib
LIB := $(LIBDIR)/libpmdfc_cceh.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
SRCS := $(CSRC)/cceh_kernels.hip $(CSRC)/bucket.hip $(CSRC)/bloom.hip $(CSRC)/ubench.hip $(CSRC)/route.hip $(CSRC)/cbf.hip $(CSRC)/trace.hip $(CSRC)/extent.hip $(CSRC)/cceh_engine.hip
HDRS := $(CSRC)/cceh_device.h $(CSRC)/cceh_kernels.h include/pmdfc_cceh.h
OBJS := $(patsubst $(CSRC)/%.hip,$(LIBDIR)/obj/%.o,$(SRCS))

HOSTLIB := $(LIBDIR)/libpmdfc_gpucceh.so
HOSTHDRS := pmdfc_amd/host/batch_core.h pmdfc_amd/host/gpu_cceh.h pmdfc_amd/host/gpu_cceh_hybrid.h pmdfc_amd/host/iface_compat.h include/pmdfc_cceh.h
KVTEST := $(LIBDIR)/test_gpu_kv
FRONTBENCH := $(LIBDIR)/bench_frontend

all: $(LIB) $(HOSTLIB) $(KVTEST) $(FRONTBENCH) oracle

$(LIBDIR)/obj/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(LIBDIR)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lrccl

$(HOSTLIB): pmdfc_amd/host/batch_core.cpp pmdfc_amd/host/kv_capi.cpp include/pmdfc_kv.h $(HOSTHDRS) $(LIB)
	$(HIPCC) -O2 -std=c++17 -fPIC -shared -Wall -o $@ pmdfc_amd/host/batch_core.cpp pmdfc_amd/host/kv_capi.cpp -L$(LIBDIR) -lpmdfc_cceh -lpthread -Wl,-rpath,'$$ORIGIN'

$(KVTEST): tests/cpp/test_gpu_kv.cpp $(HOSTLIB)
	$(HIPCC) -O2 -std=c++17 -Wall -o $@ tests/cpp/test_gpu_kv.cpp -L$(LIBDIR) -lpmdfc_gpucceh -lpmdfc_cceh -lpthread -Wl,-rpath,'$$ORIGIN'

$(FRONTBENCH): tools/bench_frontend.cpp $(HOSTLIB)
	$(HIPCC) -O2 -std=c++17 -Wall -o $@ tools/bench_frontend.cpp -L$(LIBDIR) -lpmdfc_gpucceh -lpmdfc_cceh -lpthread -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -s -C oracle liboracle.so

clean:
	rm -rf $(LIBDIR) oracle/liboracle.so

# A/B variant of the engine: make ab AB_NAME=x AB_FLAGS=-DKNOB=0 -> pmdfc_amd/lib/ab/x/libpmdfc_cceh.so
# (bench.py / tests load it with PMDFC_LIB=pmdfc_amd/lib/ab/x/libpmdfc_cceh.so)
ab:
	@mkdir -p $(LIBDIR)/ab/$(AB_NAME)/obj
	for f in $(SRCS); do $(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c -o $(LIBDIR)/ab/$(AB_NAME)/obj/$$(basename $$f .hip).o $$f || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/ab/$(AB_NAME)/libpmdfc_cceh.so $(LIBDIR)/ab/$(AB_NAME)/obj/*.o -lrccl

.PHONY: all oracle clean ab

# Top-level build of the MI355X (gfx950) SVGD library and test/bench helpers.
#   make            -> svgdcpp_amd/libsvgdcpp_amd.so (HIP kernels + C ABI, links RCCL)
#   make oracle     -> oracle/liboracle.so (CPU restatement; test infrastructure)
#   make cpp        -> build/{mvn_example,gmm_example,svgd_run_bench,test_api,test_dist} (SVGDCpp-compatible C++ API)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC_DIR := svgdcpp_amd/csrc
LIB := svgdcpp_amd/libsvgdcpp_amd.so
OBJS := $(SRC_DIR)/svgd_kernels.o $(SRC_DIR)/svgd_collect.o $(SRC_DIR)/svgd_capi.o $(SRC_DIR)/plan.o $(SRC_DIR)/host_models.o \
        $(SRC_DIR)/hostcomm.o
HDRS := $(SRC_DIR)/svgd_kernels.h $(SRC_DIR)/svgd_device.h $(SRC_DIR)/svgd_exp_table.h \
        include/svgdcpp_amd/svgd_capi.h

all: $(LIB)

$(SRC_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the matrix-core collect pass keeps its MFMA accumulators in VGPRs (gfx950's
# unified register file): no AGPR copies in its classification loop
$(SRC_DIR)/svgd_collect.o: $(SRC_DIR)/svgd_collect.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -mllvm -amdgpu-mfma-vgpr-form -c $< -o $@

$(SRC_DIR)/svgd_capi.o: $(SRC_DIR)/svgd_capi.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# host-only translation units (no device code)
$(SRC_DIR)/plan.o: $(SRC_DIR)/plan.cpp $(HDRS)
	$(CXX) -O3 -std=c++17 -fPIC -Wall -c $< -o $@

$(SRC_DIR)/hostcomm.o: $(SRC_DIR)/hostcomm.cpp $(SRC_DIR)/hostcomm.h
	$(HIPCC) -O2 -std=c++17 -fPIC -Wall -c $< -o $@

$(SRC_DIR)/host_models.o: $(SRC_DIR)/host_models.cpp $(SRC_DIR)/host_grad_block.inc $(SRC_DIR)/host_grad_soa8.inc $(HDRS)
	$(CXX) -O3 -std=c++17 -fPIC -fopenmp -Wall -Wno-psabi -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -fopenmp -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

# C++ programs over the SVGDCpp-compatible headers (include/Core, Model, Kernel, Optimizer)
CPP_FLAGS := -O2 -std=c++17 -Wall -fopenmp -Iinclude
CPP_LINK := -Lsvgdcpp_amd -lsvgdcpp_amd -Wl,-rpath,'$$ORIGIN/../svgdcpp_amd' -Wl,--allow-shlib-undefined
CPP_HDRS := $(wildcard include/SVGDCpp/*.hpp include/SVGDCpp/*/*.hpp) include/Core include/Model include/Kernel include/Optimizer
CPP_BINS := build/mvn_example build/gmm_example build/svgd_run_bench build/test_api build/test_dist

cpp: $(CPP_BINS) build/host_grad_bench

# host gradient builds side by side (tools/bench_host_grad.cpp; host only)
build/host_grad_bench: tools/bench_host_grad.cpp $(SRC_DIR)/host_models.o $(SRC_DIR)/host_models.h
	@mkdir -p build
	$(CXX) -O2 -std=c++17 -fopenmp $< $(SRC_DIR)/host_models.o -o $@

build/%: examples/%.cpp $(CPP_HDRS) $(LIB)
	@mkdir -p build
	$(CXX) $(CPP_FLAGS) $< -o $@ $(CPP_LINK)

build/test_api: tests/cpp/test_api.cpp $(CPP_HDRS) $(LIB)
	@mkdir -p build
	$(CXX) $(CPP_FLAGS) $< -o $@ $(CPP_LINK)

build/test_dist: tests/cpp/test_dist.cpp $(CPP_HDRS) $(LIB)
	@mkdir -p build
	$(CXX) $(CPP_FLAGS) $< -o $@ $(CPP_LINK)

# Host-code sanitizers (ASan + UBSan): planner, host models and the CPU oracle
# linked into a self-checking driver (the HIP host code needs a GPU: see
# tests/cpp/sanitize_host.cpp).  Run by tests/test_sanitize.py.
SAN := -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all
build/sanitize_host: tests/cpp/sanitize_host.cpp $(SRC_DIR)/plan.cpp $(SRC_DIR)/host_models.cpp oracle/svgd_oracle.c
	@mkdir -p build/san
	gcc -O1 -g -std=c11 -fopenmp -ffp-contract=off $(SAN) -c oracle/svgd_oracle.c -o build/san/oracle.o
	$(CXX) -O1 -g -std=c++17 -fopenmp $(SAN) -c $(SRC_DIR)/plan.cpp -o build/san/plan.o
	$(CXX) -O1 -g -std=c++17 -fopenmp $(SAN) -c $(SRC_DIR)/host_models.cpp -o build/san/host_models.o
	$(CXX) -O1 -g -std=c++17 -fopenmp $(SAN) tests/cpp/sanitize_host.cpp build/san/*.o -o $@ -lm

sanitize: build/sanitize_host
	ASAN_OPTIONS=detect_leaks=1 OMP_NUM_THREADS=2 ./build/sanitize_host

clean:
	rm -f $(OBJS) $(LIB) $(CPP_BINS) build/sanitize_host
	$(MAKE) -C oracle clean

.PHONY: all oracle cpp clean sanitize

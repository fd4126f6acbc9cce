# Top-level build of the MI355X (gfx950) SVGD library and test/bench helpers.
#   make            -> svgdcpp_amd/libsvgdcpp_amd.so (HIP kernels + C ABI, links RCCL)
#   make oracle     -> oracle/liboracle.so (CPU restatement; test infrastructure)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC_DIR := svgdcpp_amd/csrc
LIB := svgdcpp_amd/libsvgdcpp_amd.so
OBJS := $(SRC_DIR)/svgd_kernels.o $(SRC_DIR)/svgd_capi.o $(SRC_DIR)/plan.o $(SRC_DIR)/host_models.o
HDRS := $(SRC_DIR)/svgd_kernels.h include/svgdcpp_amd/svgd_capi.h

all: $(LIB)

$(SRC_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC_DIR)/svgd_capi.o: $(SRC_DIR)/svgd_capi.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# host-only translation units (no device code)
$(SRC_DIR)/plan.o: $(SRC_DIR)/plan.cpp $(HDRS)
	$(CXX) -O3 -std=c++17 -fPIC -Wall -c $< -o $@

$(SRC_DIR)/host_models.o: $(SRC_DIR)/host_models.cpp $(HDRS)
	$(CXX) -O3 -std=c++17 -fPIC -fopenmp -Wall -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -fopenmp -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(OBJS) $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

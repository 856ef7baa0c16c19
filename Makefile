# Build libqcart.so (HIP, gfx950) in-tree and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
PKG := deepreinforcementlearningcontrolofquantumcartpoles_amd
CSRC := $(PKG)/csrc
LIB := $(PKG)/libqcart.so
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function
OBJS := $(addprefix $(CSRC)/build/,qcart_k_ho.o qcart_k_iho.o qcart_k_grid.o qcart_dispatch.o qcart_api.o qcart_tables.o)
HDRS := include/qcart.h $(CSRC)/qcart_kargs.hpp $(CSRC)/qcart_tables.hpp $(CSRC)/qcart_kernels.hpp

all: $(LIB) oracle

$(CSRC)/build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(CSRC)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(CSRC)/build/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(CSRC)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

oracle:
	$(MAKE) -C oracle

# A/B variant: step kernel forced to a 256-VGPR budget (2 waves per SIMD)
$(PKG)/libqcart_w2.so: $(CSRC)/qcart_k_ho.hip $(CSRC)/qcart_k_iho.hip $(CSRC)/qcart_k_grid.hip $(CSRC)/qcart_dispatch.cpp $(CSRC)/qcart_api.cpp $(CSRC)/qcart_tables.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DQC_STEP_MIN_WAVES=2 -shared -o $@ $(filter %.hip %.cpp,$^)

# A/B variant: factor tables pinned in registers by LICM (the pre-reload behaviour)
$(PKG)/libqcart_pin.so: $(CSRC)/qcart_k_ho.hip $(CSRC)/qcart_k_iho.hip $(CSRC)/qcart_k_grid.hip $(CSRC)/qcart_dispatch.cpp $(CSRC)/qcart_api.cpp $(CSRC)/qcart_tables.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DQC_RELOAD_TABLES=0 -shared -o $@ $(filter %.hip %.cpp,$^)

resource-usage:
	python3 tools/kernel_resources.py $(CSRC)/build/qcart_k_*.o

clean:
	rm -rf $(CSRC)/build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean resource-usage

# Build libqcart.so (HIP, gfx950) in-tree and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
PKG := deepreinforcementlearningcontrolofquantumcartpoles_amd
CSRC := $(PKG)/csrc
LIB := $(PKG)/libqcart.so
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function
SRCS := $(CSRC)/qcart_kernels.hip $(CSRC)/qcart_api.cpp $(CSRC)/qcart_tables.cpp
HDRS := include/qcart.h $(CSRC)/qcart_kargs.hpp $(CSRC)/qcart_tables.hpp

all: $(LIB) oracle

$(CSRC)/build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(CSRC)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(CSRC)/build/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(CSRC)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(CSRC)/build/qcart_kernels.o $(CSRC)/build/qcart_api.o $(CSRC)/build/qcart_tables.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

oracle:
	$(MAKE) -C oracle

resource-usage:
	$(HIPCC) $(HIPFLAGS) -c $(CSRC)/qcart_kernels.hip -o /tmp/qcart_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS" 

clean:
	rm -rf $(CSRC)/build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean resource-usage

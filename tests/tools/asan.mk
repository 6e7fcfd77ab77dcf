# ASan + UBSan build of the path's HOST code, CPU only.
#   make -f tests/tools/asan.mk            -> build/asan/asan_host_check
# g++ compiles the C-ABI host sources (hpdct_api.cpp, hpdct_compat.cpp,
# hpdct_stream.cpp), the oracle and the check driver with the sanitizers; the
# gfx950 kernel objects of the library build are linked as they are (host
# registration stubs only; no kernel is launched: the check runs without a GPU).
# Run by tests/test_sanitizers.py in the -m "not gpu" suite.
ROOT   := $(abspath $(dir $(lastword $(MAKEFILE_LIST)))/../..)
PKG    := $(ROOT)/cuda-dct-idct_amd
OUT    := $(ROOT)/build/asan
SAN    := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
CXXF   := -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$(ROOT)/include -I$(PKG)/csrc -I$(PKG)/build $(SAN)
CF     := -std=c11 -ffp-contract=off -fno-fast-math $(SAN)
HOST   := hpdct_api hpdct_compat hpdct_stream
# the kernel objects, as the library's Makefile lists them (its KOBJ line)
PKG_KOBJ := $(filter build/%.o,$(shell sed -n 's/^KOBJ *:= *//p' $(PKG)/Makefile))
KOBJ   := $(wildcard $(PKG_KOBJ:%=$(PKG)/%))

all: $(OUT)/asan_host_check

$(OUT)/%.o: $(PKG)/csrc/%.cpp $(PKG)/csrc/hpdct_kernels.h $(PKG)/csrc/hpdct_tables.h $(ROOT)/include/hpdct.h
	@mkdir -p $(OUT)
	g++ $(CXXF) -c $< -o $@

$(OUT)/hpdct_oracle.o: $(ROOT)/oracle/hpdct_oracle.c
	@mkdir -p $(OUT)
	gcc $(CF) -c $< -o $@

$(OUT)/asan_host_check: $(ROOT)/tests/tools/asan_host_check.cpp $(PKG)/host/image_io.hpp $(HOST:%=$(OUT)/%.o) $(OUT)/hpdct_oracle.o $(KOBJ)
	g++ $(CXXF) -o $@ $< $(HOST:%=$(OUT)/%.o) $(OUT)/hpdct_oracle.o $(KOBJ) \
	    -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lpthread -lm

clean:
	rm -rf $(OUT)

.PHONY: all clean

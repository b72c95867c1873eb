# Build of the MI355X-native ALLL solver.
#   make            -> alllsatisfiabilitysolver_amd/liballl.so (HIP kernels + C-ABI, gfx950)
#   make cli        -> tools/alll_main (C++ CLI over the SATInstance compatibility headers)
#   make oracle     -> oracle/liboracle.so (test infrastructure)
#   make ref        -> oracle/_ref/ref_probe (needs /root/reference; test infrastructure)
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
ARCH ?= gfx950
PKG := alllsatisfiabilitysolver_amd
SRC := $(PKG)/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
            -Iinclude -I$(SRC) -I$(ROCM)/include $(EXTRA)
LIB := $(PKG)/liballl.so
OBJS := $(SRC)/alll_kernels.o $(SRC)/alll_stream.o $(SRC)/alll_refrng.o $(SRC)/alll_runtime.o $(SRC)/alll_host.o

all: $(LIB)

$(SRC)/alll_kernels.o: $(SRC)/alll_kernels.hip $(SRC)/alll_internal.h
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(SRC)/alll_stream.o: $(SRC)/alll_stream.hip $(SRC)/alll_internal.h
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(SRC)/alll_refrng.o: $(SRC)/alll_refrng.hip $(SRC)/alll_internal.h
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(SRC)/alll_runtime.o: $(SRC)/alll_runtime.cpp $(SRC)/alll_internal.h include/alll.h
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(SRC)/alll_host.o: $(SRC)/alll_host.cpp include/alll.h
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# (linked to a temporary name and renamed: a tree snapshot taken meanwhile sees the old or the new library)
$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@.tmp $(OBJS) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib
	mv -f $@.tmp $@

cli: tools/alll_main

tools/alll_main: tools/alll_main.cpp $(LIB) include/alll_compat/SATInstance.h
	g++ -O2 -std=c++17 -fopenmp -Iinclude/alll_compat -Iinclude -o $@ tools/alll_main.cpp \
	    -L$(PKG) -lalll -Wl,-rpath,'$$ORIGIN/../$(PKG)'

oracle:
	$(MAKE) -C oracle all

ref:
	$(MAKE) -C oracle ref

clean:
	rm -f $(OBJS) $(LIB) tools/alll_main

.PHONY: all cli oracle ref clean

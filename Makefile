# Builds the product library (HIP, gfx950) and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function
LIB := fury_amd/lib/libfory_rowfmt.so
ORACLE := oracle/_build/liboracle.so
KOBJS := fury_amd/lib/fixed.o fury_amd/lib/scan.o fury_amd/lib/varlen.o fury_amd/lib/frames.o fury_amd/lib/generic.o fury_amd/lib/treecol.o fury_amd/lib/treedec.o fury_amd/lib/launch_state.o \
         fury_amd/lib/capi.o fury_amd/lib/plan.o fury_amd/lib/host.o
HDRS := fury_amd/csrc/kernels.h fury_amd/csrc/kcommon.h fury_amd/csrc/gen_device.h fury_amd/csrc/plan.h include/fory_rowfmt.h

CAPI_TEST := tests/c/capi_roundtrip
MOCK_TEST := tests/c/host_copy_mock

all: $(LIB) $(ORACLE) $(CAPI_TEST) $(MOCK_TEST)

# The host path's copy machinery (host.cpp) on the CPU against a mock HIP runtime whose DMAs
# run late (tests/test_host_copy_mock.py): small staging blocks and registration pieces so a
# few MiB exercise reuse; host code only, under ASan + UBSan.
$(MOCK_TEST): tests/c/host_copy_mock.cpp fury_amd/csrc/host.cpp include/fory_rowfmt.h $(HDRS)
	g++ -O1 -g -std=c++17 -Wall -Wno-unused-function -D__HIP_PLATFORM_AMD__ -DFORY_STAGE_BLOCK_MB=1 -DFORY_STAGE_BLOCKS=4 \
	  -DFORY_REG_MIN_KB=64 -DFORY_REG_PIECE_KB=1024 -fsanitize=address,undefined -fno-omit-frame-pointer \
	  -I/opt/rocm/include -Ifury_amd/csrc fury_amd/csrc/host.cpp tests/c/host_copy_mock.cpp -o $@ -lpthread

# C driver of the C-ABI (GPU test tests/test_gpu_capi_c.py): plain C + HIP runtime C API
$(CAPI_TEST): tests/c/capi_roundtrip.c include/fory_rowfmt.h $(LIB) $(ORACLE)
	gcc -O2 -std=c11 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude $< -o $@ \
	  -Lfury_amd/lib -lfory_rowfmt -Loracle/_build -loracle -L/opt/rocm/lib -lamdhip64 \
	  -Wl,-rpath,'$$ORIGIN/../../fury_amd/lib:$$ORIGIN/../../oracle/_build:/opt/rocm/lib'

fury_amd/lib/%.o: fury_amd/csrc/%.hip $(HDRS)
	@mkdir -p fury_amd/lib
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

fury_amd/lib/%.o: fury_amd/csrc/%.cpp $(HDRS)
	@mkdir -p fury_amd/lib
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

$(LIB): $(KOBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(ORACLE): oracle/rowfmt_oracle.c include/fory_rowfmt.h
	@mkdir -p oracle/_build
	gcc -O2 -std=c11 -Wall -Wextra -fPIC -shared -o $@ $<

# The oracle under AddressSanitizer + UBSan (host code only), driven by the CPU tests
# that exercise it: `make asan`.
ORACLE_ASAN := oracle/_build/liboracle_asan.so
$(ORACLE_ASAN): oracle/rowfmt_oracle.c include/fory_rowfmt.h
	@mkdir -p oracle/_build
	gcc -O1 -g -std=c11 -Wall -fsanitize=address,undefined -fno-sanitize-recover=undefined \
	  -fno-omit-frame-pointer -fPIC -shared -o $@ $<

asan: $(ORACLE_ASAN)
	ORACLE_LIB=$(abspath $(ORACLE_ASAN)) LD_PRELOAD="$$(gcc -print-file-name=libasan.so) $$(gcc -print-file-name=libubsan.so)" \
	  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 python -m pytest tests/test_oracle_golden.py tests/test_infer.py -q -p no:cacheprovider

# Debug-bounds build of the library: the fixed-width kernels count
# out-of-range accesses per site and redirect them instead of faulting (fixed.hip,
# FORY_DEBUG_BOUNDS); tests select it with FORY_ROWFMT_LIB=fury_amd/lib/debug/libfory_rowfmt.so.
DEBUG_LIB := fury_amd/lib/debug/libfory_rowfmt.so
fury_amd/lib/debug/fixed.o: fury_amd/csrc/fixed.hip $(HDRS)
	@mkdir -p fury_amd/lib/debug
	$(HIPCC) $(HIPFLAGS) -DFORY_DEBUG_BOUNDS -c -o $@ $<

$(DEBUG_LIB): fury_amd/lib/debug/fixed.o $(filter-out fury_amd/lib/fixed.o,$(KOBJS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

debug: $(DEBUG_LIB)

clean:
	rm -rf fury_amd/lib oracle/_build $(CAPI_TEST)

.PHONY: all clean asan debug

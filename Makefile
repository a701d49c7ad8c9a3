# Builds the MI355X backend (libtts_hip.so, gfx950) and the CPU oracle (liboracle.so, tests only).
# No cmake: plain hipcc / gcc.  `make -j8`.

HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950

PKG := tts.cpp_amd
SRC := $(PKG)/csrc
OUT := $(PKG)/lib
OBJ := build/obj

# -ffp-contract=off: every a*b+c in the parity-relevant kernels rounds twice, as ggml's scalar C does
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
            -Wno-unused-variable -Wno-unused-but-set-variable -Wno-unused-value -Wno-unused-result -Iinclude -munsafe-fp-atomics
CXXFLAGS := -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Iinclude -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include

HIP_SRCS := $(wildcard $(SRC)/*.hip)
CPP_SRCS := $(wildcard $(SRC)/*.cpp)
HIP_OBJS := $(patsubst $(SRC)/%.hip,$(OBJ)/%.hip.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst $(SRC)/%.cpp,$(OBJ)/%.cpp.o,$(CPP_SRCS))

HARNESS := tests/ggml_stub/_build/libtts_ggml_harness.so

all: $(OUT)/libtts_hip.so oracle/_build/liboracle.so $(HARNESS)

# k_gemv: MFMA results straight into VGPRs (the Q8_0 GEMM issues a block's MFMAs back to back instead of
# funnelling each through one AGPR quad)
HIPFLAGS_k_gemv := -mllvm -amdgpu-mfma-vgpr-form

$(OBJ)/%.hip.o: $(SRC)/%.hip $(wildcard $(SRC)/*.h) include/tts_hip.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) $(HIPFLAGS_$*) -c $< -o $@

$(OBJ)/%.cpp.o: $(SRC)/%.cpp $(wildcard $(SRC)/*.h) include/tts_hip.h include/tts_runners.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -x c++ -c $< -o $@

$(OUT)/libtts_hip.so: $(HIP_OBJS) $(CPP_OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread

oracle/_build/liboracle.so: oracle/ggml_ref.c oracle/ggml_ref.h include/tts_hip.h
	$(MAKE) -C oracle

clean:
	rm -rf build $(OUT) oracle/_build

.PHONY: all clean

# Cache-policy variants of the backend for the MALL-residency study (scripts/gpu_cachepol.sh):
# lib/<variant>/libtts_hip.so, selected with TTS_HIP_LIB_VARIANT=<variant>.
VARIANT_DEFS_wplain := -DTTS_W_PLAIN
VARIANT_DEFS_kvnt := -DTTS_KV_NT
VARIANT_DEFS_wplain_kvnt := -DTTS_W_PLAIN -DTTS_KV_NT
variant-%:
	@mkdir -p build/obj_$* $(OUT)/$*
	for f in $(HIP_SRCS); do $(HIPCC) $(HIPFLAGS) $(VARIANT_DEFS_$*) -c $$f -o build/obj_$*/$$(basename $$f).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(OUT)/$*/libtts_hip.so build/obj_$*/*.hip.o $(CPP_OBJS) -lpthread
.PHONY: variant-%

# The ggml backend adapter (src/ggml_backend), compiled against the ggml fork TTS.cpp builds with
# (absent here): make ggml-adapter TTS_GGML_DIR=<checkout of mmwillet/ggml @ support-for-tts>
ggml-adapter: $(OUT)/libtts_hip.so
ifndef TTS_GGML_DIR
	$(error set TTS_GGML_DIR to a checkout of the ggml fork (mmwillet/ggml, branch support-for-tts))
endif
	g++ -std=c++17 -O2 -fPIC -shared -I$(TTS_GGML_DIR)/include -I$(TTS_GGML_DIR)/src -Iinclude -Isrc/ggml_backend \
	    src/ggml_backend/ggml-tts-hip.cpp -L$(OUT) -ltts_hip -Wl,-rpath,$(abspath $(OUT)) -o $(OUT)/libggml-tts-hip.so

# syntax / API-usage check of the adapter against declaration-only stand-ins (tests/ggml_stub)
adapter-check:
	g++ -std=c++17 -fsyntax-only -Wall -Wextra -Itests/ggml_stub -Iinclude -Isrc/ggml_backend src/ggml_backend/ggml-tts-hip.cpp

# the adapter built against the runtime stand-in (tests/ggml_stub) + a tts_backend_iface that drives its
# vtables: test infrastructure for tests/test_adapter_gpu.py (the runners run on top of the adapter)
$(HARNESS): src/ggml_backend/ggml-tts-hip.cpp src/ggml_backend/ggml-tts-hip.h $(wildcard tests/ggml_stub/*.h) \
            tests/ggml_stub/ggml_runtime.cpp tests/ggml_stub/adapter_harness.cpp include/tts_hip.h $(OUT)/libtts_hip.so
	@mkdir -p $(dir $@)
	g++ -std=c++17 -O2 -fPIC -shared -Wall -Wno-stringop-truncation -Itests/ggml_stub -Iinclude -Isrc/ggml_backend src/ggml_backend/ggml-tts-hip.cpp \
	    tests/ggml_stub/ggml_runtime.cpp tests/ggml_stub/adapter_harness.cpp -L$(OUT) -ltts_hip -Wl,-rpath,'$$ORIGIN/../../../$(OUT)' -o $@
adapter-harness: $(HARNESS)

.PHONY: ggml-adapter adapter-check adapter-harness

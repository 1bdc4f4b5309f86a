# Build of the MI355X (gfx950) SIFT hot path.
#   libsift_hip.so   -- HIP kernels + C ABI (include/sift_hip.h)
#   libsift_cuda.so  -- C++ drop-in surface sift_cuda::Detector / matchBruteForce
#                       (include/sift_cuda/*.hh), g++ only, links libsift_hip.so
#   tools            -- C++ callers mirroring the reference's tool/ examples
# The CPU oracle (test infrastructure) builds separately: make -C oracle.
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
PKG      := another-cuda-sift_amd
SRC      := $(PKG)/csrc
OUT      := $(PKG)/lib
JOBS     ?= 8
ROCM_LIB ?= /opt/rocm/lib

# -ffp-contract=off + correctly rounded f32 div/sqrt: the float operation order
# written in the kernels is the one executed (bit-exact parity with the oracle).
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -I$(SRC) -Wall -Wno-unused-result $(EXTRA_HIPFLAGS) \
            $(if $(strip $(EXTRA_HIPFLAGS)),-DSIFT_AB_FLAGS='"$(strip $(EXTRA_HIPFLAGS))"')
CXXFLAGS := -O2 -std=c++17 -fPIC -Iinclude -Wall -Wextra

HIP_SRCS := $(SRC)/detector.hip $(SRC)/lanes.hip $(SRC)/datagen.hip $(SRC)/matcher_api.hip $(SRC)/pyramid.hip $(SRC)/keypoints.hip $(SRC)/descriptor.hip $(SRC)/match.hip \
            $(SRC)/multi.hip
HIP_OBJS := $(patsubst $(SRC)/%.hip,$(OUT)/obj/%.o,$(HIP_SRCS)) $(OUT)/obj/synth_frame.o

all: $(OUT)/libsift_hip.so $(OUT)/libsift_cuda.so tools

$(OUT)/obj/%.o: $(SRC)/%.hip $(SRC)/detector_state.h $(SRC)/sift_kernels.h $(SRC)/sift_math.h $(SRC)/sift_match.h $(SRC)/sift_refine.h include/sift_hip.h
	@mkdir -p $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/obj/synth_frame.o: $(SRC)/synth_frame.cpp include/sift_hip.h
	@mkdir -p $(OUT)/obj
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OUT)/libsift_hip.so: $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS) -ldl -L$(ROCM_LIB) -lrocprofiler-sdk-roctx \
	    -Wl,-rpath,$(ROCM_LIB) -Wl,-soname,libsift_hip.so

CXX_SRCS := $(SRC)/detector_cxx.cpp $(SRC)/multi_cxx.cpp

$(OUT)/libsift_cuda.so: $(CXX_SRCS) $(wildcard include/sift_cuda/*.hh) include/sift_hip.h $(OUT)/libsift_hip.so
	$(CXX) $(CXXFLAGS) -pthread -shared -o $@ $(CXX_SRCS) -L$(OUT) -lsift_hip -Wl,-rpath,'$$ORIGIN'

tools: $(OUT)/detection_example $(OUT)/extract_and_match_example $(OUT)/multi_gpu_example $(OUT)/host_pipeline_bench

$(OUT)/%: tools/%.cpp $(OUT)/libsift_cuda.so
	$(CXX) $(CXXFLAGS) -pthread -o $@ $< -L$(OUT) -lsift_cuda -lsift_hip -Wl,-rpath,'$$ORIGIN'

# The host pipeline microbenchmark also calls the HIP runtime (pinned frames, a copy stream).
$(OUT)/host_pipeline_bench: tools/host_pipeline_bench.cpp $(OUT)/libsift_cuda.so
	$(CXX) $(CXXFLAGS) -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ $< -L$(OUT) -lsift_cuda -lsift_hip \
	    -L$(ROCM_LIB) -lamdhip64 -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(ROCM_LIB)

oracle:
	$(MAKE) -C oracle

# Sanitizer builds of the host code (HIP kernels are not
# instrumented, and GPU ASan is not available on the GPU pool): the CPU oracle,
# and the C++ drop-in surface (detector_cxx.cpp, multi_cxx.cpp) linked into the
# CPU orchestration test tests/cpp/test_multi.cpp, all with
# -fsanitize=address,undefined.  tests/test_asan.py runs both.
ASAN_DIR  := $(OUT)/asan
SANFLAGS  := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined

asan: $(ASAN_DIR)/test_multi
	$(MAKE) -C oracle asan

$(ASAN_DIR)/test_multi: tests/cpp/test_multi.cpp $(CXX_SRCS) $(wildcard include/sift_cuda/*.hh) include/sift_hip.h $(OUT)/libsift_hip.so
	@mkdir -p $(ASAN_DIR)
	$(CXX) -std=c++17 -Iinclude -Wall -Wextra $(SANFLAGS) -pthread -o $@ tests/cpp/test_multi.cpp $(CXX_SRCS) \
	    -L$(OUT) -lsift_hip -Wl,-rpath,'$$ORIGIN/..'

clean:
	rm -rf $(OUT)

.PHONY: all tools oracle asan clean

# Isolated kernel timing (tools/kernel_bench.hip), not part of `all`.
tools/kernel_bench: tools/kernel_bench.hip $(OUT)/obj/pyramid.o $(OUT)/obj/synth_frame.o
	$(HIPCC) $(HIPFLAGS) -c $< -o tools/kernel_bench.o
	$(HIPCC) --offload-arch=$(ARCH) -o $@ tools/kernel_bench.o $(OUT)/obj/pyramid.o $(OUT)/obj/synth_frame.o

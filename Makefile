# dmlc-core for MI355X — native build.
#
#   make            -> dmlc_core_amd/lib/libdmlc.so (CPU runtime + HIP kernels for gfx950)
#                      dmlc_core_amd/_dmlc*.so      (pybind11 module)
#   make test-bin   -> build/dmlc_unittest           (C++ unit tests, no GPU needed)
#   make tools      -> build/dmlc_gen, build/dmlc_bench_cpu, build/dmlc_recordio_dist,
#                      build/dmlc_fs, build/dmlc_recordio, build/dmlc_objserver
#
# Host code: g++ -std=c++17 -O3 -fopenmp -ffp-contract=off (bit-exact parsing).
# Device code: hipcc --offload-arch=gfx950 (CDNA4 only; no other targets).

ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CXX ?= g++
PYTHON ?= python3
GPU_ARCH ?= gfx950
BUILD ?= build
LIBDIR := dmlc_core_amd/lib

PY_INC := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
PY_EXT := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

WARN := -Wall -Wno-unknown-pragmas -Wno-sign-compare
CXXFLAGS_BASE := -std=c++17 -O3 -fPIC -fopenmp -ffp-contract=off -g1 $(WARN) -Iinclude -Isrc \
  -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
HIPFLAGS := -std=c++17 -O3 -fPIC --offload-arch=$(GPU_ARCH) -ffp-contract=off -Iinclude -Isrc \
  -Wno-unused-result -munsafe-fp-atomics $(HIPFLAGS_EXTRA)
LDFLAGS_LIB := -shared -fopenmp -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lrccl -ldl -lpthread

CPU_SRCS := src/logging.cc src/fault.cc src/io.cc src/recordio.cc src/data.cc src/config.cc src/synthetic.cc \
  src/io/local_filesys.cc src/io/input_split_base.cc src/io/line_split.cc \
  src/io/recordio_split.cc src/io/remote_filesys.cc \
  src/io/shard_reader.cc src/io/http.cc src/io/s3_filesys.cc src/io/azure_filesys.cc \
  src/io/hdfs_filesys.cc \
  src/gpu/runtime.cc src/gpu/device_parser.cc src/gpu/device_recordio.cc src/gpu/device_row_iter.cc \
  src/gpu/device_page_cache.cc \
  src/dist/tracker_client.cc src/dist/communicator.cc
HIP_SRCS := $(wildcard src/gpu/*.hip)

CPU_OBJS := $(patsubst src/%.cc,$(BUILD)/obj/%.o,$(CPU_SRCS))
HIP_OBJS := $(patsubst src/%.hip,$(BUILD)/obj/%.hip.o,$(HIP_SRCS))
HEADERS := $(wildcard include/dmlc/*.h include/dmlc/gpu/*.h include/dmlc/dist/*.h src/*/*.h)

LIB := $(LIBDIR)/libdmlc.so
PYMOD := dmlc_core_amd/_dmlc$(PY_EXT)

all: $(LIB) $(PYMOD)

$(BUILD)/obj/%.o: src/%.cc $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS_BASE) -c $< -o $@

$(BUILD)/obj/%.hip.o: src/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(CPU_OBJS) $(HIP_OBJS)
	@mkdir -p $(LIBDIR)
	$(CXX) -o $@ $^ $(LDFLAGS_LIB)

$(PYMOD): src/python/module.cc $(LIB) $(HEADERS)
	$(CXX) $(CXXFLAGS_BASE) -fvisibility=hidden -I$(PY_INC) -I$(PYBIND_INC) -shared \
	  src/python/module.cc -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,'$$ORIGIN/lib' \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

TEST_SRCS := $(wildcard tests/cpp/*.cc)
$(BUILD)/dmlc_unittest: $(TEST_SRCS) $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $(TEST_SRCS) -o $@ -L$(LIBDIR) -ldmlc \
	  -Wl,-rpath,$(abspath $(LIBDIR)) -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lpthread

test-bin: $(BUILD)/dmlc_unittest

# Sanitizer builds of the CPU library + unit tests: no HIP code,
# so they run anywhere.  `make tsan && build/dmlc_unittest_tsan`.
SAN_SRCS := $(filter-out src/gpu/% src/dist/communicator.cc,$(CPU_SRCS))
SAN_FLAGS := -std=c++17 -O1 -g -fno-omit-frame-pointer -ffp-contract=off $(WARN) -Iinclude -Isrc \
  -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -fopenmp
$(BUILD)/dmlc_unittest_tsan: $(TEST_SRCS) $(SAN_SRCS) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(SAN_FLAGS) -fsanitize=thread $(TEST_SRCS) $(SAN_SRCS) -o $@ -ldl -lpthread
$(BUILD)/dmlc_unittest_asan: $(TEST_SRCS) $(SAN_SRCS) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(SAN_FLAGS) -fsanitize=address,undefined $(TEST_SRCS) $(SAN_SRCS) -o $@ -ldl -lpthread
tsan: $(BUILD)/dmlc_unittest_tsan
asan: $(BUILD)/dmlc_unittest_asan

$(BUILD)/dmlc_gen: tools/dmlc_gen.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_bench_cpu: tools/dmlc_bench_cpu.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_recordio_dist: tools/dmlc_recordio_dist.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_fs: tools/dmlc_fs.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_recordio: tools/dmlc_recordio.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_parameter_example: examples/parameter.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_gpu_api_check: tools/dmlc_gpu_api_check.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

# loopback S3 / HTTP object server (sendfile) for the remote-reader benchmarks
$(BUILD)/dmlc_objserver: tools/dmlc_objserver.cc
	@mkdir -p $(BUILD)
	$(CXX) -std=c++17 -O2 -Wall -pthread $< -o $@ -lssl -lcrypto

$(BUILD)/dmlc_bench_split_cpu: tools/dmlc_bench_split_cpu.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

$(BUILD)/dmlc_bench_read: tools/dmlc_bench_read.cc $(LIB) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS_BASE) $< -o $@ -L$(LIBDIR) -ldmlc -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64

tools: $(BUILD)/dmlc_parameter_example $(BUILD)/dmlc_gen $(BUILD)/dmlc_bench_cpu $(BUILD)/dmlc_recordio_dist $(BUILD)/dmlc_fs \
  $(BUILD)/dmlc_recordio $(BUILD)/dmlc_gpu_api_check $(BUILD)/dmlc_objserver $(BUILD)/dmlc_bench_split_cpu \
  $(BUILD)/dmlc_bench_read

# same-host baseline ("re-measure on the MI355X host's CPU"): the
# reference's own sources, read in place from REF (never copied into this
# tree), built as the survey built them (-O3 -msse2 -fopenmp, no HDFS/S3), and
# this repo's public-API harnesses linked against them.  Optional: skipped when
# REF is absent.
REF ?= /root/reference
REF_SRCS := io/line_split io/indexed_recordio_split io/recordio_split io/input_split_base io \
  io/filesys io/local_filesys data recordio config
REF_OBJS := $(patsubst %,$(BUILD)/refbench/obj/%.o,$(REF_SRCS))
REF_FLAGS := -O3 -std=c++11 -msse2 -fopenmp -Wno-unknown-pragmas -DDMLC_USE_HDFS=0 -DDMLC_USE_S3=0 \
  -DDMLC_USE_AZURE=0 -I$(REF)/include
$(BUILD)/refbench/obj/%.o: $(REF)/src/%.cc
	@mkdir -p $(dir $@)
	$(CXX) $(REF_FLAGS) -c $< -o $@
$(BUILD)/refbench/ref_bench_cpu: tools/dmlc_bench_cpu.cc $(REF_OBJS)
	$(CXX) $(REF_FLAGS) $^ -o $@ -pthread
$(BUILD)/refbench/ref_bench_split_cpu: tools/dmlc_bench_split_cpu.cc $(REF_OBJS)
	$(CXX) $(REF_FLAGS) $^ -o $@ -pthread
refbench: $(BUILD)/refbench/ref_bench_cpu $(BUILD)/refbench/ref_bench_split_cpu

clean:
	rm -rf $(BUILD) $(LIB) $(PYMOD)

.PHONY: all clean test-bin tools tsan asan refbench

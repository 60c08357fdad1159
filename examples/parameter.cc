// Example: typed, self-documenting configuration with dmlc::Parameter.
//
//   ./dmlc_parameter_example chunk_mb=128 fmt=csv learning_rate=0.5
//   ./dmlc_parameter_example --help
//
// Shows defaults, ranges, enums, aliases (cf. reference example/parameter.cc,
// which demonstrates DMLC_DECLARE_ALIAS at :29-31), the error raised for an
// unknown or out-of-range key, and the JSON round trip used for checkpoints.
#include <dmlc/json.h>
#include <dmlc/logging.h>
#include <dmlc/parameter.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <vector>

struct IngestParam : public dmlc::Parameter<IngestParam> {
  int chunk_mb;
  int format;
  float learning_rate;
  std::string name;
  bool zero_copy;
  DMLC_DECLARE_PARAMETER(IngestParam) {
    DMLC_DECLARE_FIELD(chunk_mb).set_default(64).set_range(1, 4096)
        .describe("bytes per pinned / device text slot, in MiB");
    DMLC_DECLARE_FIELD(format).set_default(0)
        .add_enum("libsvm", 0).add_enum("libfm", 1).add_enum("csv", 2)
        .describe("input text format");
    DMLC_DECLARE_FIELD(learning_rate).set_default(0.1f).set_lower_bound(0.0f)
        .describe("step size of the sparse model fed by the parser");
    DMLC_DECLARE_FIELD(name).set_default("job").describe("job name");
    DMLC_DECLARE_FIELD(zero_copy).set_default(true)
        .describe("DMA straight from the page cache (mmap + hipHostRegister)");
    DMLC_DECLARE_ALIAS(format, fmt);
    DMLC_DECLARE_ALIAS(learning_rate, lr);
  }
};

DMLC_REGISTER_PARAMETER(IngestParam);

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "--help") == 0) {
    std::printf("IngestParam fields:\n%s", IngestParam::__DOC__().c_str());
    return 0;
  }
  std::vector<std::pair<std::string, std::string>> kwargs;
  for (int i = 1; i < argc; ++i) {
    const char* eq = std::strchr(argv[i], '=');
    if (eq == nullptr) continue;
    kwargs.emplace_back(std::string(argv[i], eq - argv[i]), std::string(eq + 1));
  }
  IngestParam param;
  try {
    param.Init(kwargs);
  } catch (const dmlc::ParamError& e) {
    std::fprintf(stderr, "invalid configuration: %s\n", e.what());
    return 1;
  }
  std::printf("chunk_mb=%d format=%d learning_rate=%g name=%s zero_copy=%d\n", param.chunk_mb,
              param.format, param.learning_rate, param.name.c_str(), param.zero_copy ? 1 : 0);
  // JSON round trip (what a checkpoint stores)
  std::ostringstream os;
  dmlc::JSONWriter writer(&os);
  param.Save(&writer);
  std::printf("json: %s\n", os.str().c_str());
  std::istringstream is(os.str());
  dmlc::JSONReader reader(&is);
  IngestParam copy;
  copy.Load(&reader);
  CHECK_EQ(copy.chunk_mb, param.chunk_mb);
  CHECK_EQ(copy.format, param.format);
  return 0;
}

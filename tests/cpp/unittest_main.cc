// Entry point of build/dmlc_unittest: `dmlc_unittest [--filter=Suite.] [--list]`.
#include "./testing.h"

int main(int argc, char** argv) { return testing::RunAll(argc, argv); }

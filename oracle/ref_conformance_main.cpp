// Driver for the reference's own C++ conformance tests (localTest/tests.cpp
// runTests, which also runs distribSort from localTest/benchmarks.cpp),
// compiled from the reference sources in place and linked against OUR
// libsort.so.  The reference main (localTest/main.cpp:3-22) runs the 512M-key
// benchmarks instead; this driver runs runTests(n) for each n on the command
// line.  Built by oracle/Makefile into oracle/_ref/ (test infrastructure).
#include "local.h"

#include <cstdlib>

int main(int argc, char** argv) {
  if (!initLibSort()) {
    std::cerr << "Failed to initialize libsort\n";
    return 2;
  }
  for (int i = 1; i < argc; ++i) {
    const int n = std::atoi(argv[i]);
    std::cout << "runTests(" << n << "): ";
    if (!runTests(n)) return 1;
  }
  return 0;
}

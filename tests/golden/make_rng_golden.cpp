// Golden vector for the oracle's restatement of std::mt19937 + libstdc++'s
// std::normal_distribution<float>: AdaRevisionServerTableLogic seeds one generator with
// 12345 and draws N(0, 0.1) initial row values from it
// (src/petuum_ps/server/adarevision_server_table_logic.cpp:30-34,43-46).  This program uses
// the standard library itself (not reference code); tests/test_wire_and_oracle.py builds it
// with g++ and compares its output with oracle.rng_normals bit for bit.
// usage: make_rng_golden N  -> N lines of float bits (hex)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
  std::mt19937 gen(12345);
  std::normal_distribution<float> dist(0, 0.1);
  for (int i = 0; i < n; ++i) {
    const float x = dist(gen);
    unsigned u;
    std::memcpy(&u, &x, 4);
    std::printf("%08x\n", u);
  }
  return 0;
}

// C-level single-shot latency of the liboqs-compatible entry points (no Python): median
// microseconds of OQS_KEM_keypair / encaps / decaps over N calls, one JSON line.
//   g++ -O2 -Iinclude tools/oqs_latency.cpp -Lquantum-resistant-p2p_amd/qrkem -lqrkem -Wl,-rpath,... -o oqs_latency
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "qrkem.h"

static double med(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const char* alg = argc > 1 ? argv[1] : "ML-KEM-768";
  const int N = argc > 2 ? atoi(argv[2]) : 400;
  OQS_KEM* kem = OQS_KEM_new(alg);
  if (!kem) return 1;
  std::vector<uint8_t> pk(kem->length_public_key), sk(kem->length_secret_key), ct(kem->length_ciphertext),
      ss(kem->length_shared_secret), ss2(kem->length_shared_secret);
  for (int i = 0; i < 20; ++i) OQS_KEM_keypair(kem, pk.data(), sk.data());
  using clk = std::chrono::steady_clock;
  std::vector<double> tk, te, td;
  int bad = 0;
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    OQS_KEM_keypair(kem, pk.data(), sk.data());
    auto t1 = clk::now();
    OQS_KEM_encaps(kem, ct.data(), ss.data(), pk.data());
    auto t2 = clk::now();
    OQS_KEM_decaps(kem, ss2.data(), ct.data(), sk.data());
    auto t3 = clk::now();
    bad += ss != ss2;
    tk.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    te.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
    td.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
  }
  printf("{\"alg\": \"%s\", \"c_api_median_us\": {\"keypair\": %.1f, \"encaps\": %.1f, \"decaps\": %.1f}, \"mismatches\": %d}\n",
         alg, med(tk), med(te), med(td), bad);
  OQS_KEM_free(kem);
  return bad != 0;
}

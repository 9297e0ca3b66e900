// Generates tests/golden/philox_kat.json from rocRAND's philox4x32_10 engine
// (an independent implementation of Random123's Philox4x32-10).
// engine(seed, subsequence, offset=4*k) -> first 4 outputs = Philox(ctr, key)
// with key = {seed lo, seed hi}, ctr = {k lo, k hi, subseq lo, subseq hi}.
// Build: hipcc -O1 -o /tmp/gen_kat gen_philox_kat.cpp && /tmp/gen_kat > philox_kat.json
#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>
#include <cstdint>

int main() {
  const unsigned long long seeds[] = {0ull, 0x5EEDull, 0xFFFFFFFFFFFFFFFFull,
                                      0x299f31d0a4093822ull, 1ull, 0x123456789ABCDEFull};
  const unsigned long long ks[] = {0ull, 1ull, 7ull, 0xFFFFFFFFull, 0x1234567800000009ull,
                                   0x3FFFFFFFFFFFFFFFull};
  const unsigned long long subs[] = {0ull, 1ull, 0x03000000ull | 5, 0xFFFFFFFFFFFFFFFFull,
                                     0x0800000100000002ull};
  printf("[\n");
  bool first = true;
  for (auto s : seeds)
    for (auto k : ks)
      for (auto sub : subs) {
        rocrand_device::philox4x32_10_engine eng(s, sub, 4 * k);
        unsigned int o[4];
        for (int i = 0; i < 4; ++i) o[i] = eng();
        printf("%s  {\"key\": [%u, %u], \"ctr\": [%u, %u, %u, %u], \"out\": [%u, %u, %u, %u]}",
               first ? "" : ",\n", (unsigned)s, (unsigned)(s >> 32), (unsigned)k,
               (unsigned)(k >> 32), (unsigned)sub, (unsigned)(sub >> 32), o[0], o[1], o[2], o[3]);
        first = false;
      }
  printf("\n]\n");
  return 0;
}

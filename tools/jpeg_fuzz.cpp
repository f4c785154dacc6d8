// Host JPEG decoder fuzz (ASan + UBSan build of csrc/jpeg.cpp): random byte
// edits, 0xFF / RST insertions and truncations of seed files (baseline,
// arithmetic sequential / progressive, lossless) through info, decode and
// the markers-only parse.  Seeds: files in /tmp/fz/seeds (any JPEGs).
//   g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=undefined \
//       -Imlx-data_amd/csrc -Iinclude tools/jpeg_fuzz.cpp mlx-data_amd/csrc/jpeg.cpp -o /tmp/jpeg_fuzz
#include "jpeg.h"
#include <cstdio>
#include <random>
#include <string>
#include <vector>
#include <dirent.h>
int main() {
  std::vector<std::vector<uint8_t>> seeds;
  DIR* d = opendir("/tmp/fz/seeds"); dirent* e;
  while ((e = readdir(d))) { if (e->d_name[0] == '.') continue; std::string p = std::string("/tmp/fz/seeds/") + e->d_name; FILE* f = fopen(p.c_str(), "rb"); std::vector<uint8_t> v(1 << 20); v.resize(fread(v.data(), 1, v.size(), f)); fclose(f); seeds.push_back(v); }
  closedir(d);
  std::mt19937 rng(3); long ok = 0, err = 0;
  for (int it = 0; it < 60000; it++) {
    std::vector<uint8_t> v = seeds[rng() % seeds.size()];
    int n = 1 + rng() % 8;
    for (int q = 0; q < n; q++) {
      size_t at = 2 + rng() % (v.size() - 2);
      int kind = rng() % 5;
      if (kind == 0) v[at] = rng();
      else if (kind == 1) v[at] = 0xFF;
      else if (kind == 2 && at + 1 < v.size()) { v[at] = 0xFF; v[at + 1] = 0xD0 + rng() % 8; }
      else if (kind == 3) v.resize(at);
      else v[at] ^= 1 << (rng() % 8);
      if (v.size() < 4) break;
    }
    int w = 0, h = 0, c = 0; std::string er;
    if (!mxd::jpeg::info(v.data(), v.size(), &w, &h, &c, &er)) { err++; continue; }
    if ((long)w * h > 4000000) continue;
    std::vector<uint8_t> out((size_t)w * h * 3);
    if (mxd::jpeg::decode(v.data(), v.size(), out.data(), (int64_t)w * 3, w, h, &er)) ok++; else err++;
    auto* co = mxd::jpeg::parse_coefs(v.data(), v.size(), true, &er);
    if (co) mxd::jpeg::free_coefs(co);
  }
  printf("ok %ld err %ld\n", ok, err);
}

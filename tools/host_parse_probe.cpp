// Host-side cost of a JPEG's load on the box CPU (diagnostic): per file, the
// read (open + fstat-sized read), a memcpy of the bytes, the 0xFF scan alone
// (memchr per byte found, as the marker parse does), the whole markers-only
// parse (mxd::jpeg::parse_coefs), load_coefs (read + parse) and unstuff().
//   g++ -O2 -std=c++17 -Imlx-data_amd/csrc -Iinclude tools/host_parse_probe.cpp mlx-data_amd/csrc/jpeg.cpp \
//       -o tools/host_parse_probe && tools/host_parse_probe DIR_OF_JPEGS
#include "jpeg.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::vector<std::string> paths;
  DIR* d = opendir(argv[1]);
  if (!d) return 2;
  while (dirent* e = readdir(d))
    if (strstr(e->d_name, ".jpg")) paths.push_back(std::string(argv[1]) + "/" + e->d_name);
  closedir(d);
  std::vector<std::vector<uint8_t>> files;
  for (auto& p : paths) {
    FILE* f = fopen(p.c_str(), "rb");
    std::vector<uint8_t> v(1 << 22);
    v.resize(fread(v.data(), 1, v.size(), f));
    fclose(f);
    files.push_back(v);
  }
  std::vector<uint8_t> dst(1 << 22);
  const int reps = 30;
  const char* names[6] = {"read", "memcpy", "ff_scan", "parse", "load", "unstuff"};
  for (int mode = 0; mode < 6; mode++) {
    const double t0 = now_us();
    long sink = 0;
    for (int r = 0; r < reps; r++)
      for (size_t i = 0; i < files.size(); i++) {
        const auto& v = files[i];
        if (mode == 0) {
          const int fd = open(paths[i].c_str(), O_RDONLY);
          struct stat st;
          fstat(fd, &st);
          std::vector<uint8_t> b((size_t)st.st_size);
          sink += read(fd, b.data(), b.size());
          close(fd);
        } else if (mode == 1) {
          std::memcpy(dst.data(), v.data(), v.size());
          sink += dst[v.size() / 2];
        } else if (mode == 2) {
          size_t p = 0;
          for (;;) {
            const void* f = memchr(v.data() + p, 0xFF, v.size() - p);
            if (!f) break;
            p = (size_t)(static_cast<const uint8_t*>(f) - v.data()) + 1;
            sink++;
          }
        } else if (mode == 3) {
          auto* c = mxd::jpeg::parse_coefs(v.data(), v.size(), true, nullptr);
          mxd::jpeg::free_coefs(c);
        } else if (mode == 4) {
          bool nj = false;
          auto* c = mxd::jpeg::load_coefs(paths[i].c_str(), true, &nj, nullptr);
          mxd::jpeg::free_coefs(c);
        } else {
          sink += mxd::jpeg::unstuff(v.data() + 700, v.data() + v.size() - 2, dst.data());
        }
      }
    printf("{\"probe\": \"%s\", \"us_per_file\": %.2f, \"files\": %zu, \"sink\": %ld}\n", names[mode],
           (now_us() - t0) / (reps * files.size()), files.size(), sink & 1);
  }
  return 0;
}

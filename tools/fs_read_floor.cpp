// Floor of the fs ingest on this host: lstat / open+fstat+close / open+fstat+pread+close of
// every regular file of a tree, from T threads (tools/gpu_fs_floor.sh).  usage: fs_read_floor DIR T MODE
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>
#include <thread>
#include <atomic>
#include <cstring>
int main(int argc, char** argv) {
  std::vector<std::string> files, dirs{argv[1]};
  for (size_t i = 0; i < dirs.size(); i++) {
    DIR* d = opendir(dirs[i].c_str());
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      std::string p = dirs[i] + "/" + e->d_name;
      if (e->d_type == DT_DIR) dirs.push_back(p); else if (e->d_type == DT_REG) files.push_back(p);
    }
    closedir(d);
  }
  int T = atoi(argv[2]); int mode = atoi(argv[3]);
  for (int rep = 0; rep < 5; rep++) {
    std::atomic<size_t> next{0}; std::atomic<uint64_t> tot{0};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back([&] {
      std::vector<char> buf(1 << 20);
      for (;;) {
        size_t i = next.fetch_add(8); if (i >= files.size()) break;
        for (size_t k = i; k < std::min(files.size(), i + 8); k++) {
          struct stat st;
          if (mode == 0) { lstat(files[k].c_str(), &st); continue; }
          int fd = open(files[k].c_str(), O_RDONLY);
          fstat(fd, &st);
          if (mode == 2) { size_t n = std::min<size_t>(st.st_size, buf.size()); ssize_t r = pread(fd, buf.data(), n, 0); tot += r; }
          close(fd);
        }
      }
    });
    for (auto& x : th) x.join();
    printf("mode %d T %d: %.1f ms (%zu files, %lu bytes)\n", mode, T, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), files.size(), (unsigned long)tot.load());
  }
}

// Host <-> device copy paths for the host-memory API forms (DESIGN.md,
// end-to-end rates): pageable hipMemcpy, hipHostRegister of the caller's
// buffer, and threaded memcpy into pinned staging.  Build:
//   hipcc -O2 -std=c++17 -o tools/host_copy_probe tools/host_copy_probe.cpp -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(void *dst, const void *src, size_t bytes, int threads) {
  std::vector<std::thread> t;
  const size_t per = (bytes / threads + 4095) & ~(size_t)4095;
  for (int i = 0; i < threads; ++i) {
    const size_t a = (size_t)i * per;
    if (a >= bytes) break;
    const size_t b = a + per < bytes ? a + per : bytes;
    t.emplace_back([=] { memcpy((char *)dst + a, (const char *)src + a, b - a); });
  }
  for (auto &x : t) x.join();
}

int main(int argc, char **argv) {
  const size_t bytes = (size_t)(argc > 1 ? atof(argv[1]) : 4.0) * (1ull << 30);
  const double gib = bytes / double(1ull << 30);
  char *h = (char *)malloc(bytes), *h2 = (char *)malloc(bytes);
  memset(h, 1, bytes);
  memset(h2, 2, bytes);
  void *d = nullptr, *pin = nullptr;
  if (hipMalloc(&d, bytes) || hipHostMalloc(&pin, bytes, hipHostMallocDefault)) return 1;
  memset(pin, 0, bytes);
  double t;
  for (int rep = 0; rep < 2; ++rep) {
    t = now();
    hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    printf("pageable H2D        %7.1f GiB/s\n", gib / (now() - t));
    t = now();
    hipMemcpy(h2, d, bytes, hipMemcpyDeviceToHost);
    printf("pageable D2H        %7.1f GiB/s\n", gib / (now() - t));
    t = now();
    hipMemcpy(d, pin, bytes, hipMemcpyHostToDevice);
    printf("pinned H2D          %7.1f GiB/s\n", gib / (now() - t));
    t = now();
    hipMemcpy(pin, d, bytes, hipMemcpyDeviceToHost);
    printf("pinned D2H          %7.1f GiB/s\n", gib / (now() - t));
    t = now();
    hipHostRegister(h, bytes, hipHostRegisterDefault);
    const double tr = now() - t;
    void *dh = nullptr;
    hipHostGetDevicePointer(&dh, h, 0);
    double t2 = now();
    hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    const double tc = now() - t2;
    t2 = now();
    hipHostUnregister(h);
    const double tu = now() - t2;
    printf("register %5.1f GiB/s, registered H2D %5.1f GiB/s, unregister %5.1f GiB/s, all %5.1f GiB/s\n",
           gib / tr, gib / tc, gib / tu, gib / (tr + tc + tu));
    for (int th : {1, 4, 8, 16, 32}) {
      t = now();
      par_copy(pin, h, bytes, th);
      printf("memcpy -> pinned x%-2d %7.1f GiB/s\n", th, gib / (now() - t));
    }
  }
  return 0;
}

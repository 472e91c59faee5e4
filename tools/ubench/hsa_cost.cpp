// Where the HIP runtime's start-up goes below hipInit (tools/ubench/init_cost.hip
// measures hipInit as one 120-256 ms block): the raw KFD open, loading the
// HSA runtime library, hsa_init() and the agent walk, each timed in a fresh
// process.  No GPU work is submitted.
//
//   g++ -O2 -I/opt/rocm/include tools/ubench/hsa_cost.cpp -ldl -o tools/ubench/hsa_cost
//   tools/ubench/hsa_cost            # one JSON line of milliseconds
#include <dlfcn.h>
#include <fcntl.h>
#include <hsa/hsa.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

using init_fn = hsa_status_t (*)();
using iter_fn = hsa_status_t (*)(hsa_status_t (*)(hsa_agent_t, void*), void*);

static hsa_status_t count_agent(hsa_agent_t, void* n) {
  ++*static_cast<int*>(n);
  return HSA_STATUS_SUCCESS;
}

int main() {
  double t = now_ms();
  const int fd = open("/dev/kfd", O_RDWR | O_CLOEXEC);
  const double kfd_open = now_ms() - t;
  if (fd >= 0) close(fd);
  t = now_ms();
  void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  const double dl = now_ms() - t;
  if (!h) {
    std::printf("{\"error\": \"dlopen: %s\"}\n", dlerror());
    return 1;
  }
  auto hsa_init_p = reinterpret_cast<init_fn>(dlsym(h, "hsa_init"));
  auto hsa_shut_p = reinterpret_cast<init_fn>(dlsym(h, "hsa_shut_down"));
  auto hsa_iter_p = reinterpret_cast<iter_fn>(dlsym(h, "hsa_iterate_agents"));
  t = now_ms();
  const hsa_status_t st = hsa_init_p();
  const double init = now_ms() - t;
  int agents = 0;
  t = now_ms();
  if (st == HSA_STATUS_SUCCESS) hsa_iter_p(count_agent, &agents);
  const double iter = now_ms() - t;
  t = now_ms();
  if (st == HSA_STATUS_SUCCESS) hsa_shut_p();
  const double shut = now_ms() - t;
  std::printf("{\"kfd_open_ms\": %.3f, \"dlopen_hsa_ms\": %.3f, \"hsa_init_ms\": %.3f, \"status\": %d, "
              "\"agents\": %d, \"iterate_ms\": %.3f, \"shutdown_ms\": %.3f}\n",
              kfd_open, dl, init, static_cast<int>(st), agents, iter, shut);
  return 0;
}

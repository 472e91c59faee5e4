// HIP runtime RAII wrappers (see device.hpp).
#include "pconv/device.hpp"

#include <dlfcn.h>
#include <sched.h>

#include <cctype>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace pconv {

int device_count() {
  int n = 0;
  PCONV_HIP_CHECK(hipGetDeviceCount(&n));
  return n;
}

void set_device(int device) {
  const int n = device_count();
  PCONV_CHECK(device >= 0 && device < n,
              "device " + std::to_string(device) + " out of range (" + std::to_string(n) + " visible)");
  PCONV_HIP_CHECK(hipSetDevice(device));
}

std::string device_pci_bus_id(int device) {
  char buf[64] = {0};
  PCONV_HIP_CHECK(hipDeviceGetPCIBusId(buf, static_cast<int>(sizeof(buf)), device));
  std::string id(buf);
  for (auto& c : id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return id;
}

HipRuntimeInfo hip_runtime_info() {
  HipRuntimeInfo r;
  PCONV_HIP_CHECK(hipRuntimeGetVersion(&r.runtime_version));
  (void)hipDriverGetVersion(&r.driver_version);
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&hipRuntimeGetVersion), &info) != 0 && info.dli_fname) {
    r.runtime_path = info.dli_fname;
    // the symbol's address may be this library's PLT stub: resolve the real
    // definition through the global scope instead
    if (void* real = dlsym(RTLD_DEFAULT, "hipRuntimeGetVersion"))
      if (dladdr(real, &info) != 0 && info.dli_fname) r.runtime_path = info.dli_fname;
  }
  r.compiled_version = std::to_string(HIP_VERSION_MAJOR) + "." + std::to_string(HIP_VERSION_MINOR) + "." +
                       std::to_string(HIP_VERSION_PATCH);
  return r;
}

int bind_to_device_numa(int device) {
  const char* env = std::getenv("PCONV_NUMA_BIND");
  if (env && std::string(env) == "0") return 0;
  std::ifstream f("/sys/bus/pci/devices/" + device_pci_bus_id(device) + "/local_cpulist");
  std::string text;
  if (!f || !std::getline(f, text)) return 0;
  cpu_set_t allowed, keep;
  CPU_ZERO(&keep);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return 0;
  std::stringstream ss(text);
  std::string part;
  while (std::getline(ss, part, ',')) {
    if (part.empty()) continue;
    const auto dash = part.find('-');
    const int a = std::stoi(part.substr(0, dash));
    const int b = dash == std::string::npos ? a : std::stoi(part.substr(dash + 1));
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, &keep);
  }
  const int n = CPU_COUNT(&keep);
  if (n == 0 || CPU_EQUAL(&keep, &allowed)) return 0;
  return sched_setaffinity(0, sizeof(keep), &keep) == 0 ? n : 0;
}

std::string device_name(int device) {
  hipDeviceProp_t p;
  PCONV_HIP_CHECK(hipGetDeviceProperties(&p, device));
  return std::string(p.name) + " (" + p.gcnArchName + ")";
}

DeviceBuffer::DeviceBuffer(size_t bytes) : bytes_(bytes) {
  if (bytes) {
    void* p = nullptr;
    PCONV_HIP_CHECK(hipMalloc(&p, bytes));
    ptr_ = static_cast<uint8_t*>(p);
  }
}

DeviceBuffer::~DeviceBuffer() {
  if (ptr_) (void)hipFree(ptr_);
}

DeviceBuffer& DeviceBuffer::operator=(DeviceBuffer&& o) noexcept {
  std::swap(ptr_, o.ptr_);
  std::swap(bytes_, o.bytes_);
  return *this;
}

PinnedBuffer::PinnedBuffer(size_t bytes) : bytes_(bytes) {
  if (bytes) {
    void* p = nullptr;
    PCONV_HIP_CHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
    ptr_ = static_cast<uint8_t*>(p);
  }
}

PinnedBuffer::~PinnedBuffer() {
  if (ptr_) (void)hipHostFree(ptr_);
}

PinnedBuffer& PinnedBuffer::operator=(PinnedBuffer&& o) noexcept {
  std::swap(ptr_, o.ptr_);
  std::swap(bytes_, o.bytes_);
  return *this;
}

Stream Stream::create(int priority) {
  Stream s;
  PCONV_HIP_CHECK(hipStreamCreateWithPriority(&s.s_, hipStreamNonBlocking, priority));
  return s;
}

Stream::~Stream() {
  if (s_) (void)hipStreamDestroy(s_);
}

void Stream::sync() const { PCONV_HIP_CHECK(hipStreamSynchronize(s_)); }

Event Event::create(bool timing) {
  Event e;
  PCONV_HIP_CHECK(hipEventCreateWithFlags(&e.e_, timing ? hipEventDefault : hipEventDisableTiming));
  return e;
}

Event::~Event() {
  if (e_) (void)hipEventDestroy(e_);
}

void Event::record(hipStream_t s) const { PCONV_HIP_CHECK(hipEventRecord(e_, s)); }
void Event::wait_on(hipStream_t s) const { PCONV_HIP_CHECK(hipStreamWaitEvent(s, e_, 0)); }
void Event::sync() const { PCONV_HIP_CHECK(hipEventSynchronize(e_)); }

float Event::elapsed_ms(const Event& a, const Event& b) {
  float ms = 0.f;
  PCONV_HIP_CHECK(hipEventElapsedTime(&ms, a.e_, b.e_));
  return ms;
}

}  // namespace pconv

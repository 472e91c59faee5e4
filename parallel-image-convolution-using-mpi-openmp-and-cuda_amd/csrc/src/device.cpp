// HIP runtime RAII wrappers (see device.hpp).
#include "pconv/device.hpp"

#include <dlfcn.h>
#include <sched.h>

#include <algorithm>
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

double copy_pair_floor_ms(int device, int64_t row_bytes, int64_t rows_in, int64_t rows_out, int iters) {
  PCONV_CHECK(row_bytes > 0 && rows_in > 0 && rows_out > 0 && iters > 0, "copy_pair_floor_ms: empty copy");
  set_device(device);
  const int64_t pitch = (row_bytes + 16 + 127) / 128 * 128;  // a padded frame pitch like the engine's
  DeviceBuffer din(static_cast<size_t>(pitch * rows_in)), dout(static_cast<size_t>(pitch * rows_out));
  PinnedBuffer hin(static_cast<size_t>(row_bytes * rows_in)), hout(static_cast<size_t>(row_bytes * rows_out));
  Stream s1 = Stream::create(0), s2 = Stream::create(0);
  Event e0 = Event::create(true), a = Event::create(true), b = Event::create(true);
  auto pairs = [&](int n) {
    PCONV_HIP_CHECK(hipDeviceSynchronize());
    e0.record(s1.get());
    e0.wait_on(s2.get());
    for (int i = 0; i < n; ++i) {
      PCONV_HIP_CHECK(hipMemcpy2DAsync(din.data() + 16, static_cast<size_t>(pitch), hin.data(),
                                       static_cast<size_t>(row_bytes), static_cast<size_t>(row_bytes),
                                       static_cast<size_t>(rows_in), hipMemcpyHostToDevice, s1.get()));
      PCONV_HIP_CHECK(hipMemcpy2DAsync(hout.data(), static_cast<size_t>(row_bytes), dout.data() + 16,
                                       static_cast<size_t>(pitch), static_cast<size_t>(row_bytes),
                                       static_cast<size_t>(rows_out), hipMemcpyDeviceToHost, s2.get()));
    }
    a.record(s1.get());
    b.record(s2.get());
    a.sync();
    b.sync();
    return std::max(Event::elapsed_ms(e0, a), Event::elapsed_ms(e0, b)) / n;
  };
  (void)pairs(2);  // warm: first-use queue / engine set-up
  return std::min(pairs(iters), pairs(iters));
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

DeviceBuffer::DeviceBuffer(size_t bytes, unsigned flags) : bytes_(bytes) {
  if (bytes) {
    void* p = nullptr;
    PCONV_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, flags));
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

Stream Stream::create_cu_masked(const std::vector<uint32_t>& mask) {
  Stream s;
  PCONV_HIP_CHECK(hipExtStreamCreateWithCUMask(&s.s_, static_cast<uint32_t>(mask.size()), mask.data()));
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

// Resident convolution service (see service.hpp).
#include "pconv/service.hpp"

#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstring>
#include <memory>

#include "pconv/common.hpp"
#include "pconv/device.hpp"

namespace pconv {

namespace {

constexpr uint32_t kMaxArgs = 256;
constexpr uint32_t kMaxArgBytes = 1 << 16;
constexpr uint32_t kMaxReplyBytes = 1 << 24;

// Whole-buffer socket I/O with a deadline (poll between partial transfers).
void io_all(int fd, void* buf, size_t n, bool writing, double deadline) {
  auto* p = static_cast<uint8_t*>(buf);
  while (n > 0) {
    const double left = deadline - wall_seconds();
    PCONV_CHECK(left > 0, "service: timed out");
    pollfd pf{fd, static_cast<short>(writing ? POLLOUT : POLLIN), 0};
    const int pr = ::poll(&pf, 1, static_cast<int>(std::min(left, 1e6) * 1000) + 1);
    if (pr < 0 && errno == EINTR) continue;
    PCONV_CHECK(pr >= 0, std::string("service: poll: ") + std::strerror(errno));
    if (pr == 0) continue;
    const ssize_t k = writing ? ::send(fd, p, n, MSG_NOSIGNAL) : ::recv(fd, p, n, 0);
    if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    PCONV_CHECK(k > 0, k == 0 ? "service: peer closed the connection"
                              : std::string("service: ") + std::strerror(errno));
    p += k;
    n -= static_cast<size_t>(k);
  }
}

void send_u32(int fd, uint32_t v, double dl) { io_all(fd, &v, sizeof(v), true, dl); }
uint32_t recv_u32(int fd, double dl) {
  uint32_t v = 0;
  io_all(fd, &v, sizeof(v), false, dl);
  return v;
}

sockaddr_un address(const std::string& path) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  PCONV_CHECK(!path.empty() && path.size() < sizeof(a.sun_path), "service: socket path empty or too long");
  std::memcpy(a.sun_path, path.c_str(), path.size() + 1);
  return a;
}

struct Fd {
  int fd = -1;
  explicit Fd(int f) : fd(f) {}
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

}  // namespace

ServeOptions parse_serve_args(const std::vector<std::string>& args) {
  ServeOptions o;
  PCONV_CHECK(args.size() >= 3 && args[1] == "--serve", "usage: conv --serve SOCKET [options]");
  o.socket_path = args[2];
  for (size_t i = 3; i < args.size(); ++i) {
    auto val = [&](const char* what) -> std::string {
      PCONV_CHECK(i + 1 < args.size(), std::string("missing value for ") + what);
      return args[++i];
    };
    if (args[i] == "--device") o.device = std::stoi(val("--device"));
    else if (args[i] == "--idle-timeout") o.idle_timeout_s = std::stod(val("--idle-timeout"));
    else if (args[i] == "--max-engines") o.max_engines = std::stoi(val("--max-engines"));
    else PCONV_FAIL("unknown serve option '" + args[i] + "'");
  }
  PCONV_CHECK(o.device >= -1 && o.max_engines >= 1 && o.idle_timeout_s >= 0, "bad serve options");
  return o;
}

int serve_main(const ServeOptions& o) {
  // The device first: a server that cannot reach its GPU never listens.
  // --device -1: a CPU-only server (the cpu / omp backends).
  if (o.device >= 0) {
    set_device(o.device);
    PCONV_HIP_CHECK(hipFree(nullptr));
  }
  std::unique_ptr<JobCache, void (*)(JobCache*)> cache(new_job_cache(o.device, o.max_engines), delete_job_cache);

  Fd ls(::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0));
  PCONV_CHECK(ls.fd >= 0, std::string("service: socket: ") + std::strerror(errno));
  const sockaddr_un addr = address(o.socket_path);
  // A leftover socket of a dead server is replaced; anything else at that
  // path (a regular file, a live server) is refused, never deleted.
  struct stat st{};
  if (::lstat(o.socket_path.c_str(), &st) == 0) {
    PCONV_CHECK(S_ISSOCK(st.st_mode), "service: " + o.socket_path + " exists and is not a socket");
    Fd probe(::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0));
    PCONV_CHECK(probe.fd >= 0 && ::connect(probe.fd, reinterpret_cast<const sockaddr*>(&addr), sizeof(addr)) != 0,
                "service: a server is already listening on " + o.socket_path);
    ::unlink(o.socket_path.c_str());
  }
  const mode_t old = ::umask(077);  // owner-only socket
  const int br = ::bind(ls.fd, reinterpret_cast<const sockaddr*>(&addr), sizeof(addr));
  ::umask(old);
  PCONV_CHECK(br == 0, "service: bind " + o.socket_path + ": " + std::strerror(errno));
  PCONV_CHECK(::listen(ls.fd, 16) == 0, std::string("service: listen: ") + std::strerror(errno));
  std::fprintf(stderr, "conv: serving on %s (device %d)\n", o.socket_path.c_str(), o.device);
  std::fflush(stderr);

  int jobs = 0;
  bool stop = false;
  double last = wall_seconds();
  while (!stop) {
    pollfd pf{ls.fd, POLLIN, 0};
    const int pr = ::poll(&pf, 1, 500);
    if (pr < 0 && errno == EINTR) continue;
    PCONV_CHECK(pr >= 0, std::string("service: poll: ") + std::strerror(errno));
    if (pr == 0) {
      if (o.idle_timeout_s > 0 && wall_seconds() - last > o.idle_timeout_s) break;
      continue;
    }
    Fd cfd(::accept4(ls.fd, nullptr, nullptr, SOCK_CLOEXEC));
    if (cfd.fd < 0) continue;
    const double dl = wall_seconds() + 30.0;  // request transfer deadline
    std::string reply;
    try {
      const uint32_t argc = recv_u32(cfd.fd, dl);
      PCONV_CHECK(argc >= 1 && argc <= kMaxArgs, "service: bad request");
      std::vector<std::string> args(argc);
      for (auto& a : args) {
        const uint32_t n = recv_u32(cfd.fd, dl);
        PCONV_CHECK(n <= kMaxArgBytes, "service: argument too long");
        a.resize(n);
        if (n) io_all(cfd.fd, a.data(), n, false, dl);
      }
      if (args[0] == "__shutdown__") {
        reply = "{\"ok\": true, \"jobs\": " + std::to_string(jobs) + "}";
        stop = true;
      } else if (args[0] == "__ping__") {
        reply = "{\"ok\": true, \"jobs\": " + std::to_string(jobs) + ", \"device\": " + std::to_string(o.device) +
                "}";
      } else {
        CliConfig c = parse_cli(args);
        PCONV_CHECK(c.server.empty(), "service: a job cannot name another server");
        PCONV_CHECK(o.device >= 0 || c.backend != Backend::Hip, "service: this server has no GPU (--device -1)");
        const AppReport r = run_app(c, cache.get());
        reply = report_json(c, r);
        ++jobs;
      }
    } catch (const std::exception& e) {
      reply = std::string("{\"error\": \"") + json_escape(e.what()) + "\"}";
    }
    try {
      send_u32(cfd.fd, static_cast<uint32_t>(reply.size()), wall_seconds() + 30.0);
      io_all(cfd.fd, reply.data(), reply.size(), true, wall_seconds() + 30.0);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "conv serve: reply failed: %s\n", e.what());
    }
    last = wall_seconds();
  }
  if (::lstat(o.socket_path.c_str(), &st) == 0 && S_ISSOCK(st.st_mode)) ::unlink(o.socket_path.c_str());
  return 0;
}

std::string service_request(const std::string& socket_path, const std::vector<std::string>& args,
                            double timeout_s) {
  Fd fd(::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0));
  PCONV_CHECK(fd.fd >= 0, std::string("service: socket: ") + std::strerror(errno));
  const sockaddr_un addr = address(socket_path);
  PCONV_CHECK(::connect(fd.fd, reinterpret_cast<const sockaddr*>(&addr), sizeof(addr)) == 0,
              "service: connect " + socket_path + ": " + std::strerror(errno) + " (is `conv --serve` running?)");
  const double dl = wall_seconds() + timeout_s;
  PCONV_CHECK(args.size() <= kMaxArgs, "service: too many arguments");
  send_u32(fd.fd, static_cast<uint32_t>(args.size()), dl);
  for (const auto& a : args) {
    PCONV_CHECK(a.size() <= kMaxArgBytes, "service: argument too long");
    send_u32(fd.fd, static_cast<uint32_t>(a.size()), dl);
    if (!a.empty()) io_all(fd.fd, const_cast<char*>(a.data()), a.size(), true, dl);
  }
  const uint32_t n = recv_u32(fd.fd, dl);
  PCONV_CHECK(n <= kMaxReplyBytes, "service: reply too long");
  std::string reply(n, '\0');
  if (n) io_all(fd.fd, reply.data(), n, false, dl);
  return reply;
}

}  // namespace pconv

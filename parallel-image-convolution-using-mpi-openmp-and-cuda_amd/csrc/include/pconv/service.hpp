// Resident convolution service: a warm GPU context behind a unix socket.
//
// The reference is a one-shot program whose end-to-end timer
// (cuda/main.c:20-49) includes CUDA context creation; on MI355X the HIP
// runtime's start-up alone (hipInit + the first hardware queue, 140-270 ms on
// the boxes measured, profiles/r02/) is larger than the reference's smallest
// GTX 970 cells.  For serving many images, `conv --serve SOCKET` initialises
// the device ONCE and then executes jobs sent by thin clients:
//
//   conv --serve /tmp/pconv.sock [--device D] [--idle-timeout S]   (server)
//   conv image.raw W H reps rgb --server /tmp/pconv.sock [flags]   (client)
//
// A job is the client's argv (image / --out made absolute); the server parses
// it with the same CLI contract, reads the file, runs it on its cached engine
// (device frames, pinned staging, tuned kernels and graphs kept per geometry),
// writes the output and answers with the report JSON.  The client prints the
// reference's timing lines itself, timing from after its argument parsing to
// the answer — the same bracket as the reference, HIP init excluded because
// the context is already up.  One job at a time (jobs on one GPU serialise
// anyway); 1 GPU, or the CPU backends.
//
// Wire format (host byte order, same machine): request = u32 argc, then per
// argument u32 length + bytes; reply = u32 length + JSON bytes.  argv[0] of
// "__shutdown__" stops the server; "__ping__" answers {"ok": true}.
#pragma once

#include <string>
#include <vector>

#include "pconv/app.hpp"

namespace pconv {

struct ServeOptions {
  std::string socket_path;
  int device = 0;
  double idle_timeout_s = 0;  // 0: serve until a shutdown request
  int max_engines = 8;        // cached engines (LRU)
};

// Runs the server loop; returns the process exit code.
int serve_main(const ServeOptions& o);

// Client side: send `args` (argv[0] included) to the server and return the
// reply JSON.  Throws on connection / protocol errors.
std::string service_request(const std::string& socket_path, const std::vector<std::string>& args,
                            double timeout_s = 600.0);

// Parse `conv --serve ...` options (args[1] == "--serve").
ServeOptions parse_serve_args(const std::vector<std::string>& args);

}  // namespace pconv

// Python bindings (pybind11) for the native engine: module `_pconv_native`.
//
// Buffers cross the boundary either as Python buffer-protocol objects (numpy
// arrays, host memory) or as raw integer addresses (torch.Tensor.data_ptr()
// of CUDA tensors or pinned host tensors) — no torch C++ ABI dependency.
#include <omp.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "pconv/app.hpp"
#include "pconv/cpu_stencil.hpp"
#include "pconv/device.hpp"
#include "pconv/engine.hpp"
#include "pconv/ipc_halo.hpp"
#include "pconv/kernels.hpp"
#include "pconv/partition.hpp"
#include "pconv/selftest.hpp"
#include "pconv/raw_io.hpp"
#include "pconv/rccl_comm.hpp"
#include "pconv/schedule.hpp"
#include "../kernels/swar.hpp"

namespace py = pybind11;
using namespace pconv;

namespace {

struct HostView {
  uint8_t* ptr;
  int64_t size;
};

HostView host_view(py::buffer b, bool writable) {
  py::buffer_info info = b.request(writable);
  PCONV_CHECK(info.itemsize == 1, "expected a uint8 buffer");
  // Must be C-contiguous.
  int64_t expect = 1;
  for (int i = info.ndim - 1; i >= 0; --i) {
    PCONV_CHECK(info.strides[i] == expect, "expected a C-contiguous buffer");
    expect *= info.shape[i];
  }
  return {static_cast<uint8_t*>(info.ptr), static_cast<int64_t>(info.size)};
}

ImageGeom make_geom(int64_t w, int64_t h, const std::string& ch) {
  ImageGeom g;
  g.width = w;
  g.height = h;
  g.channels = parse_channels(ch);
  g.validate();
  return g;
}

KernelVariant parse_variant(const std::string& s) {
  if (s == "auto") return KernelVariant::Auto;
  if (s == "binomial") return KernelVariant::Binomial;
  if (s == "temporal") return KernelVariant::Temporal;
  if (s == "int9") return KernelVariant::Int9;
  if (s == "float9") return KernelVariant::Float9;
  if (s == "float_temporal") return KernelVariant::FloatTemporal;
  PCONV_FAIL("unknown kernel variant '" + s + "'");
}

Filter make_filter(py::object f) {
  if (py::isinstance<py::str>(f)) return Filter::by_name(f.cast<std::string>());
  return f.cast<Filter>();
}

// Halo transport implemented in Python (e.g. host-staged gloo messages for
// several ranks sharing one GPU in tests).  The Python subclass implements
// exchange_rows(row0_ptr, pitch, rows, up, down, depth, stream): fill ghost
// rows [-depth, 0) / [rows, rows+depth) of the frame whose owned row 0 starts
// at row0_ptr (pitch-aligned, pads included) and send the matching owned rows,
// enqueued on (or synchronised with) `stream`.
class PyHaloTransport : public HaloTransport {
 public:
  void exchange(BandEngine& e, int64_t depth, hipStream_t stream) override {
    py::gil_scoped_acquire gil;
    py::function f = py::get_override(static_cast<const HaloTransport*>(this), "exchange_rows");
    PCONV_CHECK(static_cast<bool>(f), "HaloTransport subclass must implement exchange_rows()");
    f(reinterpret_cast<uintptr_t>(e.src_frame() - kPadLeft), e.layout().pitch, e.band().rows, e.band().up,
      e.band().down, depth, reinterpret_cast<uintptr_t>(stream));
  }
  const char* name() const override { return "python"; }
};

}  // namespace

PYBIND11_MODULE(_pconv_native, m) {
  m.doc() = "pconv native engine: CDNA4 HIP stencil kernels, HIP runtime, RCCL halos, CPU oracle";

  py::register_exception<Error>(m, "NativeError", PyExc_RuntimeError);

  // ---------------------------------------------------------------- filters
  py::class_<Filter>(m, "Filter")
      .def_static("gaussian", &Filter::gaussian)
      .def_static("box", &Filter::box)
      .def_static("edge", &Filter::edge)
      .def_static("by_name", &Filter::by_name)
      .def_static("custom", &Filter::custom, py::arg("taps"), py::arg("divisor"), py::arg("name") = "custom")
      .def_readonly("name", &Filter::name)
      .def_readonly("taps", &Filter::taps)
      .def_readonly("divisor", &Filter::divisor)
      .def_readonly("weights", &Filter::weights)
      .def_readonly("int_exact", &Filter::int_exact)
      .def_readonly("shift", &Filter::shift)
      .def_readonly("binomial121", &Filter::binomial121)
      .def("__repr__", [](const Filter& f) { return "Filter(" + f.name + "/" + std::to_string(f.divisor) + ")"; });

  // ---------------------------------------------------------------- geometry
  m.def(
      "frame_layout",
      [](int64_t row_bytes, int64_t rows, int64_t halo) {
        const FrameLayout l = FrameLayout::make(row_bytes, rows, halo);
        return py::dict(py::arg("row_bytes") = l.row_bytes, py::arg("rows") = l.rows, py::arg("halo") = l.halo,
                        py::arg("pitch") = l.pitch, py::arg("bytes") = l.bytes(), py::arg("pad_left") = kPadLeft);
      },
      py::arg("row_bytes"), py::arg("rows"), py::arg("halo"));

  py::class_<Band>(m, "Band")
      .def(py::init<>())
      .def_readwrite("rank", &Band::rank)
      .def_readwrite("world", &Band::world)
      .def_readwrite("y0", &Band::y0)
      .def_readwrite("rows", &Band::rows)
      .def_readwrite("up", &Band::up)
      .def_readwrite("down", &Band::down)
      .def("__repr__", [](const Band& b) {
        return "Band(rank=" + std::to_string(b.rank) + ", y0=" + std::to_string(b.y0) + ", rows=" +
               std::to_string(b.rows) + ", up=" + std::to_string(b.up) + ", down=" + std::to_string(b.down) + ")";
      });
  m.def("row_band", &row_band, py::arg("height"), py::arg("world"), py::arg("rank"));
  m.def("row_bands", &row_bands, py::arg("height"), py::arg("world"));
  m.def("reference_rows_division", &reference_rows_division);

  // ---------------------------------------------------------------- schedule
  py::class_<LaunchSpec>(m, "LaunchSpec")
      .def_readonly("steps", &LaunchSpec::steps)
      .def_readonly("lo", &LaunchSpec::lo)
      .def_readonly("hi", &LaunchSpec::hi)
      .def_readonly("after_halo", &LaunchSpec::after_halo);
  py::class_<Phase>(m, "Phase")
      .def_readonly("exchange_depth", &Phase::exchange_depth)
      .def_readonly("steps", &Phase::steps)
      .def_readonly("launches", &Phase::launches);
  m.def(
      "plan_band",
      [](const Band& b, int reps, int halo_depth, int fuse, bool overlap, bool halo_preloaded) {
        PlanConfig c;
        c.halo_depth = halo_depth;
        c.fuse = fuse;
        c.overlap = overlap;
        c.halo_preloaded = halo_preloaded;
        return plan_band(b, reps, c);
      },
      py::arg("band"), py::arg("reps"), py::arg("halo_depth") = 1, py::arg("fuse") = 1, py::arg("overlap") = true,
      py::arg("halo_preloaded") = false);
  m.def(
      "normalize_plan",
      [](int halo_depth, int fuse, int64_t min_band_rows, int max_fuse) {
        PlanConfig c;
        c.halo_depth = halo_depth;
        c.fuse = fuse;
        c = normalize_plan_config(c, min_band_rows, max_fuse);
        return py::make_tuple(c.halo_depth, c.fuse);
      },
      py::arg("halo_depth"), py::arg("fuse"), py::arg("min_band_rows"), py::arg("max_fuse") = kMaxFusedSteps);
  m.def("describe_plan", &describe_plan);
  m.attr("MAX_FUSED_STEPS") = kMaxFusedSteps;
  py::class_<StreamChunk>(m, "StreamChunk")
      .def_readonly("up_lo", &StreamChunk::up_lo)
      .def_readonly("up_hi", &StreamChunk::up_hi)
      .def_readonly("launches", &StreamChunk::launches)
      .def_readonly("levels", &StreamChunk::levels)
      .def_readonly("down_lo", &StreamChunk::down_lo)
      .def_readonly("down_hi", &StreamChunk::down_hi);
  py::class_<StreamPlan>(m, "StreamPlan")
      .def_readonly("levels", &StreamPlan::levels)
      .def_readonly("chunks", &StreamPlan::chunks);
  m.def("streamable", &streamable, py::arg("plan"));
  m.def("stream_cuts", &stream_cuts, py::arg("in_lo"), py::arg("in_hi"), py::arg("chunks"));
  m.def("stream_cuts_weighted", &stream_cuts_weighted, py::arg("in_lo"), py::arg("in_hi"), py::arg("weights"));
  m.def("plan_streamed", &plan_streamed, py::arg("plan"), py::arg("in_lo"), py::arg("in_hi"), py::arg("owned_rows"),
        py::arg("cuts"));

  // ---------------------------------------------------------------- CPU oracle
  m.def(
      "cpu_convolve",
      [](py::buffer in, py::buffer out, int64_t w, int64_t h, const std::string& ch, int reps, py::object filter,
         bool omp, int threads) {
        const ImageGeom g = make_geom(w, h, ch);
        const HostView a = host_view(in, false), b = host_view(out, true);
        PCONV_CHECK(a.size == g.bytes() && b.size == g.bytes(), "buffer size does not match the image geometry");
        const Filter f = make_filter(filter);
        py::gil_scoped_release nogil;
        cpu_convolve(f, g, a.ptr, b.ptr, reps, omp ? CpuBackend::OpenMP : CpuBackend::Serial, threads);
      },
      py::arg("src"), py::arg("dst"), py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("reps"),
      py::arg("filter") = "gaussian", py::arg("omp") = false, py::arg("threads") = 0);
  m.def("default_cpu_threads", &default_cpu_threads,
        "OpenMP team size used when none is set: affinity CPUs capped by the cgroup quota, minus one");
  m.def(
      "set_cpu_threads",
      [](int n) {
        omp_set_num_threads(std::max(1, n));
        return omp_get_max_threads();
      },
      py::arg("n"), "OpenMP team size of this process's CPU stencil (returns the size now in effect)");
  m.def("cpu_threads", []() { return omp_get_max_threads(); }, "OpenMP team size in effect");
  m.def("configure_cpu_threads", &configure_cpu_threads, py::arg("share") = 1,
        "Size the OpenMP team (unless OMP_NUM_THREADS is set) for `share` processes on this node");
  m.def(
      "cpu_fused_launch",
      [](py::object filter, const std::string& ch, int64_t row_bytes, int64_t rows, int64_t halo, py::buffer src,
         py::buffer dst, int64_t lo, int64_t hi, int steps, int64_t g_row0, int64_t height, bool omp) {
        const FrameLayout lay = FrameLayout::make(row_bytes, rows, halo);
        const HostView a = host_view(src, false), b = host_view(dst, true);
        PCONV_CHECK(a.size == lay.bytes() && b.size == lay.bytes(), "frame buffer size mismatch");
        const Filter f = make_filter(filter);
        py::gil_scoped_release nogil;
        cpu_fused_launch(f, parse_channels(ch), lay, a.ptr, b.ptr, lo, hi, steps, g_row0, height,
                         omp ? CpuBackend::OpenMP : CpuBackend::Serial);
      },
      py::arg("filter"), py::arg("channels"), py::arg("row_bytes"), py::arg("rows"), py::arg("halo"), py::arg("src"),
      py::arg("dst"), py::arg("lo"), py::arg("hi"), py::arg("steps"), py::arg("g_row0"), py::arg("height"),
      py::arg("omp") = false);

  // ---------------------------------------------------------------- raw I/O
  m.def("output_path_for", &output_path_for, py::arg("path"), py::arg("prefix") = "blur_");
  m.def(
      "read_raw",
      [](const std::string& path, py::buffer dst, int64_t w, int64_t h, const std::string& ch) {
        const ImageGeom g = make_geom(w, h, ch);
        const HostView b = host_view(dst, true);
        PCONV_CHECK(b.size == g.bytes(), "buffer size does not match the image geometry");
        read_image(path, g, b.ptr);
      },
      py::arg("path"), py::arg("dst"), py::arg("width"), py::arg("height"), py::arg("channels"));
  m.def(
      "read_raw_rows",
      [](const std::string& path, py::buffer dst, int64_t w, int64_t h, const std::string& ch, int64_t y0,
         int64_t rows) {
        const ImageGeom g = make_geom(w, h, ch);
        const HostView b = host_view(dst, true);
        PCONV_CHECK(b.size >= rows * g.row_bytes(), "buffer too small");
        validate_input_file(path, g);
        read_rows(path, g, y0, rows, b.ptr, g.row_bytes());
      },
      py::arg("path"), py::arg("dst"), py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("y0"),
      py::arg("rows"));
  m.def(
      "write_raw",
      [](const std::string& path, py::buffer src, int64_t w, int64_t h, const std::string& ch) {
        const ImageGeom g = make_geom(w, h, ch);
        const HostView b = host_view(src, false);
        PCONV_CHECK(b.size == g.bytes(), "buffer size does not match the image geometry");
        write_image(path, g, b.ptr);
      },
      py::arg("path"), py::arg("src"), py::arg("width"), py::arg("height"), py::arg("channels"));
  m.def(
      "create_output",
      [](const std::string& path, int64_t w, int64_t h, const std::string& ch) {
        create_output(path, make_geom(w, h, ch));
      },
      py::arg("path"), py::arg("width"), py::arg("height"), py::arg("channels"));
  m.def(
      "write_raw_rows",
      [](const std::string& path, py::buffer src, int64_t w, int64_t h, const std::string& ch, int64_t y0,
         int64_t rows) {
        const ImageGeom g = make_geom(w, h, ch);
        const HostView b = host_view(src, false);
        PCONV_CHECK(b.size >= rows * g.row_bytes(), "buffer too small");
        write_rows(path, g, y0, rows, b.ptr, g.row_bytes());
      },
      py::arg("path"), py::arg("src"), py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("y0"),
      py::arg("rows"));
  m.def(
      "synth_rows",
      [](py::buffer dst, int64_t w, int64_t h, const std::string& ch, uint64_t seed, int64_t y0, int64_t rows) {
        const ImageGeom g = make_geom(w, h, ch);
        const HostView b = host_view(dst, true);
        PCONV_CHECK(b.size >= rows * g.row_bytes(), "buffer too small");
        py::gil_scoped_release nogil;
        synth_rows(g, seed, y0, rows, b.ptr, g.row_bytes());
      },
      py::arg("dst"), py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("seed"), py::arg("y0"),
      py::arg("rows"));

  // ---------------------------------------------------------------- CLI
  m.def("conv_main", [](std::vector<std::string> argv) {
    std::vector<char*> ptrs;
    for (auto& s : argv) ptrs.push_back(s.data());
    py::gil_scoped_release nogil;
    return conv_main(static_cast<int>(ptrs.size()), ptrs.data());
  });

  // ---------------------------------------------------------------- device
  m.def("device_count", &device_count);
  m.def("device_name", &device_name);
  m.def("set_device", &set_device);
  m.def("device_pci_bus_id", &device_pci_bus_id);
  m.def("copy_pair_floor_ms", &copy_pair_floor_ms, py::arg("device"), py::arg("row_bytes"), py::arg("rows_in"),
        py::arg("rows_out"), py::arg("iters") = 8,
        "ms per pitched H2D + D2H pair issued concurrently on two streams (the pipeline's PCIe floor)");
  m.def(
      "page_nodes", [](uintptr_t p, size_t bytes) { return page_nodes(reinterpret_cast<const void*>(p), bytes); },
      py::arg("ptr"), py::arg("bytes"), "NUMA node -> pages of a host range (move_pages query; negative: -errno)");
  m.def("device_numa_node", &device_numa_node, py::arg("device"));
  m.def(
      "flush_host_cache",
      [](uintptr_t p, size_t bytes) {
        py::gil_scoped_release nogil;
        flush_host_cache(reinterpret_cast<const void*>(p), bytes);
      },
      py::arg("ptr"), py::arg("bytes"), "clflush a host range out of every CPU cache (staging written by the CPU)");
  m.def(
      "copy_floor_on",
      [](int device, uintptr_t host_in, uintptr_t host_out, int64_t row_bytes, int64_t rows_in, int64_t rows_out,
         int iters) {
        py::gil_scoped_release nogil;
        const CopyFloor f = copy_floor_on(device, reinterpret_cast<uint8_t*>(host_in),
                                          reinterpret_cast<uint8_t*>(host_out), row_bytes, rows_in, rows_out, iters);
        return std::make_tuple(f.h2d_ms, f.d2h_ms, f.pair_ms);
      },
      py::arg("device"), py::arg("host_in"), py::arg("host_out"), py::arg("row_bytes"), py::arg("rows_in"),
      py::arg("rows_out"), py::arg("iters") = 8,
      "(H2D alone, D2H alone, concurrent pair) ms with the given pinned host buffers (0: fresh ones)");
  py::class_<CopyProbe>(m, "CopyProbe")
      .def(py::init([](int device, int64_t row_bytes, int64_t rows_in, int64_t rows_out) {
             py::gil_scoped_release nogil;
             return std::make_unique<CopyProbe>(device, nullptr, nullptr, row_bytes, rows_in, rows_out);
           }),
           py::arg("device"), py::arg("row_bytes"), py::arg("rows_in"), py::arg("rows_out"))
      .def("run", &CopyProbe::run, py::arg("n"), py::arg("up") = true, py::arg("down") = true,
           py::call_guard<py::gil_scoped_release>(),
           "ms per copy (pair) over n pitched H2D and / or D2H copies issued on two streams");
  m.def("bind_to_device_numa", &bind_to_device_numa,
        "Restrict this process to the CPUs local to the GPU (returns the CPUs kept; 0: unchanged)");

  py::class_<PinnedBuffer>(m, "PinnedBuffer", py::buffer_protocol())
      .def(py::init<size_t>())
      .def_property_readonly("ptr", [](const PinnedBuffer& b) { return reinterpret_cast<uintptr_t>(b.data()); })
      .def("__len__", &PinnedBuffer::size)
      .def_buffer([](PinnedBuffer& b) -> py::buffer_info {
        return py::buffer_info(b.data(), 1, py::format_descriptor<uint8_t>::format(), 1,
                               {static_cast<py::ssize_t>(b.size())}, {1});
      });

  m.def(
      "launch_stencil",
      [](py::object filter, const std::string& ch, uintptr_t src, uintptr_t dst, int64_t pitch, int64_t row_bytes,
         int64_t r0, int64_t r1, int64_t frame_lo, int64_t frame_hi, int steps, int64_t g_row0, int64_t height,
         uintptr_t stream, const std::string& variant) {
        StencilLaunch a;
        a.src = reinterpret_cast<const uint8_t*>(src);
        a.dst = reinterpret_cast<uint8_t*>(dst);
        a.pitch = pitch;
        a.row_bytes = row_bytes;
        a.r0 = r0;
        a.r1 = r1;
        a.frame_lo = frame_lo;
        a.frame_hi = frame_hi;
        a.steps = steps;
        a.g_row0 = g_row0;
        a.height = height;
        launch_stencil(make_filter(filter), parse_channels(ch), a, reinterpret_cast<hipStream_t>(stream),
                       parse_variant(variant));
      },
      py::arg("filter"), py::arg("channels"), py::arg("src"), py::arg("dst"), py::arg("pitch"), py::arg("row_bytes"),
      py::arg("r0"), py::arg("r1"), py::arg("frame_lo"), py::arg("frame_hi"), py::arg("steps") = 1,
      py::arg("g_row0") = 0, py::arg("height") = (int64_t(1) << 40), py::arg("stream") = 0,
      py::arg("variant") = "auto");
  m.def("set_swar_shape", &set_swar_shape, py::arg("lw") = 0, py::arg("m") = 0, py::arg("nw") = 0,
        "Force the SWAR temporal tile shape (lw=0: back to the latency model).");
  m.def("swar_shapes", []() {
    py::list out;
    for (const auto& s : swar_shapes()) out.append(py::make_tuple(s.lw, s.m, s.nw));
    return out;
  });
  m.def(
      "swar_model",
      [](int steps, const std::string& ch, int64_t rows, int64_t row_bytes) {
        const SwarShape s = pick_swar_shape(steps, channel_count(parse_channels(ch)), rows, row_bytes);
        return py::make_tuple(py::make_tuple(s.lw, s.m, s.nw),
                              swar_launch_cycles(s, steps, channel_count(parse_channels(ch)), rows, row_bytes));
      },
      py::arg("steps"), py::arg("channels"), py::arg("rows"), py::arg("row_bytes"));
  m.def("set_autotune", &set_autotune, py::arg("on"),
        "Time the model's best SWAR tile shapes on first use of a launch geometry (default on).");
  m.def("clear_swar_tuning", &clear_swar_tuning);
  m.def("swar_tuned", []() {
    py::list out;
    for (const auto& kv : swar_tuned())
      out.append(py::make_tuple(py::cast(kv.first), py::make_tuple(kv.second.lw, kv.second.m, kv.second.nw)));
    return out;
  });
  m.def("set_prefetch_mode", &set_prefetch_mode, py::arg("mode"),
        "Buffer-op tile kernel: -1 tuned against the others (default), 0 never, 1 forced (with a set_swar_shape "
        "shape it instantiates, that shape)");
  m.def("set_tune_candidates", &set_tune_candidates, py::arg("n"),
        "How many of the latency model's best SWAR tile shapes the tuner times (default 6).");
  m.def("set_float_shape", &set_float_shape, py::arg("m") = 0, py::arg("nw") = 0,
        "Force the float temporal kernel's tile (m rows per wave, nw waves; m=0: model / tuner).");
  m.def("swar_prefetch_shapes", []() {
    py::list out;
    for (const auto& s : swar_prefetch_shapes()) out.append(py::make_tuple(s.lw, s.m, s.nw));
    return out;
  });
  m.def("set_swar_alt", &set_swar_alt, py::arg("mode"),
        "SWAR step form: -1 tuned (default), 0 truncate every step, 1 pairs of steps with a x16 intermediate.");
  m.def("set_xcd_swizzle", &set_xcd_swizzle, py::arg("on"),
        "XCD-aware (bijective, per-XCD contiguous) tile order of the SWAR kernel.");
  m.def(
      "swar_model_table",
      [](int steps, const std::string& ch, int64_t rows, int64_t row_bytes) {
        // every shape: (lw, m, nw, vgpr, lds, measured, predicted cycles)
        const int c = channel_count(parse_channels(ch));
        py::list out;
        for (const auto& s : swar_shapes()) {
          const SwarResources r = swar_resources(s, c);
          out.append(py::make_tuple(s.lw, s.m, s.nw, r.vgpr, r.lds, r.measured,
                                    swar_launch_cycles(s, steps, c, rows, row_bytes)));
        }
        return out;
      },
      py::arg("steps"), py::arg("channels"), py::arg("rows"), py::arg("row_bytes"));
  m.def("auto_fuse",
        [](py::object filter, const std::string& v, int64_t frame_bytes, int channels) {
          return auto_fuse(make_filter(filter), parse_variant(v), frame_bytes, channels);
        },
        py::arg("filter"), py::arg("variant"), py::arg("frame_bytes"), py::arg("channels") = 0,
        "Default repetitions per launch for a band frame of `frame_bytes` with `channels` bytes per pixel");
  m.def("supports_fusion",
        [](py::object filter, const std::string& v) { return supports_fusion(make_filter(filter), parse_variant(v)); },
        py::arg("filter"), py::arg("variant") = "auto");

  // ---------------------------------------------------------------- engine
  py::class_<RunStats>(m, "RunStats")
      .def_readonly("loop_ms", &RunStats::loop_ms)
      .def_readonly("wall_ms", &RunStats::wall_ms)
      .def_readonly("launches", &RunStats::launches)
      .def_readonly("exchanges", &RunStats::exchanges);

  py::class_<HaloTransport, PyHaloTransport, std::shared_ptr<HaloTransport>>(m, "HaloTransport")
      .def(py::init<>())
      .def_property_readonly("name", &HaloTransport::name);

  m.def(
      "memcpy_async",
      [](uintptr_t dst, uintptr_t src, int64_t nbytes, const std::string& kind, uintptr_t stream) {
        hipMemcpyKind k = kind == "h2d" ? hipMemcpyHostToDevice
                          : kind == "d2h" ? hipMemcpyDeviceToHost
                          : kind == "d2d" ? hipMemcpyDeviceToDevice
                                          : hipMemcpyDefault;
        PCONV_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src),
                                       static_cast<size_t>(nbytes), k, reinterpret_cast<hipStream_t>(stream)));
      },
      py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("kind"), py::arg("stream") = 0);
  m.def(
      "stream_synchronize",
      [](uintptr_t stream) { PCONV_HIP_CHECK(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream))); },
      py::arg("stream"), py::call_guard<py::gil_scoped_release>());

  py::class_<BandEngine>(m, "BandEngine")
      .def(py::init([](int64_t w, int64_t h, const std::string& ch, py::object filter, int rank, int world,
                       int device, int halo, int fuse, bool overlap, bool graph, const std::string& variant,
                       bool kernel_copies, int stream_chunks) {
             EngineOptions o;
             o.stream_chunks = stream_chunks;
             o.kernel_copies = kernel_copies;
             o.device = device;
             o.halo_depth = halo;
             o.fuse = fuse;
             o.overlap = overlap;
             o.use_graph = graph;
             o.variant = parse_variant(variant);
             const ImageGeom g = make_geom(w, h, ch);
             return std::make_unique<BandEngine>(g, row_band(h, world, rank), make_filter(filter), o);
           }),
           py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("filter") = "gaussian",
           py::arg("rank") = 0, py::arg("world") = 1, py::arg("device") = 0, py::arg("halo") = 1, py::arg("fuse") = 1,
           py::arg("overlap") = true, py::arg("graph") = false, py::arg("variant") = "auto",
           py::arg("kernel_copies") = false, py::arg("stream_chunks") = 0)
      .def_property_readonly("band", &BandEngine::band)
      .def("stream_plan", &BandEngine::stream_plan, py::arg("reps"), py::arg("in_r0"), py::arg("in_r1"))
      .def_property_readonly("halo", [](const BandEngine& e) { return e.layout().halo; })
      .def_property_readonly("fuse", [](const BandEngine& e) { return e.options().fuse; })
      .def_property_readonly("cached_graphs", &BandEngine::cached_graphs)
      .def_property_readonly("cached_step_graphs", &BandEngine::cached_step_graphs)
      .def_property_readonly_static("max_cached_graphs", [](py::object) { return BandEngine::kMaxCachedGraphs; })
      .def_property_readonly("pitch", [](const BandEngine& e) { return e.layout().pitch; })
      .def_property_readonly("row_bytes", [](const BandEngine& e) { return e.layout().row_bytes; })
      .def_property_readonly("compute_stream",
                             [](const BandEngine& e) { return reinterpret_cast<uintptr_t>(e.compute_stream()); })
      .def_property_readonly("comm_stream",
                             [](const BandEngine& e) { return reinterpret_cast<uintptr_t>(e.comm_stream()); })
      .def_property_readonly("src_ptr", [](const BandEngine& e) { return reinterpret_cast<uintptr_t>(e.src_frame()); })
      .def("plan", &BandEngine::plan, py::arg("reps"))
      .def(
          "upload",
          [](BandEngine& e, py::buffer host, int64_t r_begin, int64_t r_end) {
            const HostView v = host_view(host, false);
            PCONV_CHECK(v.size >= (r_end - r_begin) * e.layout().row_bytes, "host buffer too small");
            e.upload_rows(v.ptr, e.layout().row_bytes, r_begin, r_end);
          },
          py::arg("host"), py::arg("r_begin"), py::arg("r_end"))
      .def(
          "upload_ptr",
          [](BandEngine& e, uintptr_t ptr, int64_t pitch, int64_t r_begin, int64_t r_end, bool device) {
            if (device)
              e.upload_rows_device(reinterpret_cast<const uint8_t*>(ptr), pitch, r_begin, r_end);
            else
              e.upload_rows(reinterpret_cast<const uint8_t*>(ptr), pitch, r_begin, r_end);
          },
          py::arg("ptr"), py::arg("pitch"), py::arg("r_begin"), py::arg("r_end"), py::arg("device") = false)
      .def(
          "download",
          [](BandEngine& e, py::buffer host, int64_t r_begin, int64_t r_end) {
            const HostView v = host_view(host, true);
            PCONV_CHECK(v.size >= (r_end - r_begin) * e.layout().row_bytes, "host buffer too small");
            e.download_rows(v.ptr, e.layout().row_bytes, r_begin, r_end);
          },
          py::arg("host"), py::arg("r_begin"), py::arg("r_end"))
      .def(
          "download_ptr",
          [](BandEngine& e, uintptr_t ptr, int64_t pitch, int64_t r_begin, int64_t r_end, bool device) {
            if (device)
              e.download_rows_device(reinterpret_cast<uint8_t*>(ptr), pitch, r_begin, r_end);
            else
              e.download_rows(reinterpret_cast<uint8_t*>(ptr), pitch, r_begin, r_end);
          },
          py::arg("ptr"), py::arg("pitch"), py::arg("r_begin"), py::arg("r_end"), py::arg("device") = false)
      .def("set_halo_valid", &BandEngine::set_halo_valid)
      .def("wait_stream", [](BandEngine& e, uintptr_t s) { e.wait_stream(reinterpret_cast<hipStream_t>(s)); })
      .def("signal_stream", [](BandEngine& e, uintptr_t s) { e.signal_stream(reinterpret_cast<hipStream_t>(s)); })
      .def("run", &BandEngine::run, py::arg("reps"), py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &BandEngine::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("clear", &BandEngine::clear)
      .def_property_readonly("stats", &BandEngine::last_stats)
      .def(
          "process",
          [](BandEngine& e, uintptr_t in_ptr, int64_t in_r0, int64_t in_r1, uintptr_t out_ptr, int reps) {
            // Serving step: H2D (rows [in_r0, in_r1), ghost rows allowed), reps, D2H of
            // the owned rows; host pointers pinned.  Releases the GIL throughout.
            py::gil_scoped_release nogil;
            const int64_t rb = e.layout().row_bytes;
            e.upload_rows(reinterpret_cast<const uint8_t*>(in_ptr), rb, in_r0, in_r1);
            e.set_halo_valid(in_r0 < 0 || in_r1 > e.band().rows);
            e.run(reps);
            e.download_rows(reinterpret_cast<uint8_t*>(out_ptr), rb, 0, e.band().rows);
            e.synchronize();
          },
          py::arg("in_ptr"), py::arg("in_r0"), py::arg("in_r1"), py::arg("out_ptr"), py::arg("reps"))
      .def(
          "process_graph",
          [](BandEngine& e, uintptr_t in_ptr, int64_t in_r0, int64_t in_r1, uintptr_t out_ptr, int reps) {
            py::gil_scoped_release nogil;
            e.process_graph(reinterpret_cast<const uint8_t*>(in_ptr), in_r0, in_r1, reinterpret_cast<uint8_t*>(out_ptr),
                            reps);
          },
          py::arg("in_ptr"), py::arg("in_r0"), py::arg("in_r1"), py::arg("out_ptr"), py::arg("reps"))
      .def("exchange_free", &BandEngine::exchange_free, py::arg("reps"), py::arg("halo_preloaded"))
      .def("input_preloaded", &BandEngine::input_preloaded, py::arg("in_r0"), py::arg("in_r1"))
      .def(
          "exchange_now",
          [](BandEngine& e, uintptr_t stream) { e.exchange_now(reinterpret_cast<hipStream_t>(stream)); },
          py::arg("stream") = 0, "Fill the whole ghost zone now (transport on `stream`, 0 = the comm stream)")
      .def(
          "read_frame",
          [](BandEngine& e, py::buffer host, int64_t r_begin, int64_t r_end) {
            const HostView v = host_view(host, true);
            PCONV_CHECK(v.size >= (r_end - r_begin) * e.layout().row_bytes, "host buffer too small");
            py::gil_scoped_release nogil;
            e.read_frame_rows(v.ptr, r_begin, r_end);
          },
          py::arg("host"), py::arg("r_begin"), py::arg("r_end"),
          "Copy source-frame rows [r_begin, r_end), ghost rows included (tests / debugging)")
      .def_static(
          "for_band",
          [](int64_t w, int64_t h, const std::string& ch, py::object filter, const Band& band, int device, int halo,
             int fuse, bool overlap, const std::string& variant, bool graph, bool capture_exchanges) {
            // An explicit band (tests: e.g. a single rank whose up/down
            // neighbour is itself, to drive RCCL send/recv-to-self).
            EngineOptions o;
            o.device = device;
            o.halo_depth = halo;
            o.fuse = fuse;
            o.overlap = overlap;
            o.variant = parse_variant(variant);
            o.use_graph = graph;
            o.capture_exchanges = capture_exchanges;
            return std::make_unique<BandEngine>(make_geom(w, h, ch), band, make_filter(filter), o);
          },
          py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("filter"), py::arg("band"),
          py::arg("device") = 0, py::arg("halo") = 1, py::arg("fuse") = 1, py::arg("overlap") = true,
          py::arg("variant") = "auto", py::arg("graph") = false, py::arg("capture_exchanges") = false)
      .def("set_stream_trace", &BandEngine::set_stream_trace, py::arg("on"),
           "diagnostics: time the next streamed images chunk by chunk (stream_trace())")
      .def("stream_trace", &BandEngine::stream_trace, py::call_guard<py::gil_scoped_release>(),
           "latest streamed image: [chunk, upload end, launches end, download end] ms from its start")
      .def("attach_rccl",
           [](BandEngine& e, std::shared_ptr<RcclComm> c) {
             e.set_transport(std::make_shared<RcclTransport>(std::move(c)));
           })
      .def("attach_transport", [](BandEngine& e, std::shared_ptr<HaloTransport> t) { e.set_transport(std::move(t)); },
           py::keep_alive<1, 2>())
      .def("attach_null_transport",
           [](BandEngine& e) { e.set_transport(std::make_shared<NullTransport>()); });

  py::class_<BandPipeline>(m, "BandPipeline")
      .def(py::init([](int64_t w, int64_t h, const std::string& ch, py::object filter, int rank, int world,
                       int device, int halo, int fuse, bool overlap, const std::string& variant, int slots,
                       int concurrent, bool graphs, bool step_graphs, py::object band, bool slot_comm,
                       int stream_chunks, bool cu_mask_queues, bool head_on_slot_streams,
                       int64_t stream_min_bytes, bool head_alt_uploads, std::vector<int> stream_weights,
                       bool lazy_head) {
             EngineOptions o;
             o.lazy_head = lazy_head;
             o.head_alt_uploads = head_alt_uploads;
             o.stream_chunks = stream_chunks;
             PCONV_CHECK(stream_weights.empty() || static_cast<int>(stream_weights.size()) == stream_chunks,
                         "stream_weights: one weight per chunk (stream_chunks of them)");
             o.stream_weights = std::move(stream_weights);
             o.stream_min_bytes = stream_min_bytes;
             o.cu_mask_queues = cu_mask_queues;
             o.head_on_slot_streams = head_on_slot_streams;
             o.device = device;
             o.halo_depth = halo;
             o.fuse = fuse;
             o.overlap = overlap;
             o.variant = parse_variant(variant);
             const ImageGeom g = make_geom(w, h, ch);
             // band: an explicit Band (tests: a self-neighbour band on a 1-rank communicator)
             const Band b = band.is_none() ? row_band(h, world, rank) : band.cast<Band>();
             return std::make_unique<BandPipeline>(g, b, make_filter(filter), o, slots, concurrent, graphs,
                                                   step_graphs, slot_comm);
           }),
           py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("filter") = "gaussian",
           py::arg("rank") = 0, py::arg("world") = 1, py::arg("device") = 0, py::arg("halo") = 1, py::arg("fuse") = 1,
           py::arg("overlap") = true, py::arg("variant") = "auto", py::arg("slots") = 2, py::arg("concurrent") = -1,
           py::arg("graphs") = false, py::arg("step_graphs") = true,
           py::arg("band") = py::none(), py::arg("slot_comm") = false, py::arg("stream_chunks") = 0,
           py::arg("cu_mask_queues") = true, py::arg("head_on_slot_streams") = true,
           py::arg("stream_min_bytes") = EngineOptions{}.stream_min_bytes, py::arg("head_alt_uploads") = true,
           py::arg("stream_weights") = std::vector<int>{}, py::arg("lazy_head") = EngineOptions{}.lazy_head)
      .def_property_readonly("slots", &BandPipeline::slots)
      .def("slot", &BandPipeline::slot, py::return_value_policy::reference_internal)
      .def("attach_rccl",
           [](BandPipeline& p, std::shared_ptr<RcclComm> c) {
             p.set_transport(std::make_shared<RcclTransport>(std::move(c)));
           })
      .def("attach_transport", [](BandPipeline& p, std::shared_ptr<HaloTransport> t) { p.set_transport(std::move(t)); },
           py::keep_alive<1, 2>())
      .def("attach_slot_rccl",
           [](BandPipeline& p, int k, std::shared_ptr<RcclComm> c) {
             p.set_slot_transport(k, std::make_shared<RcclTransport>(std::move(c)));
           })
      .def("attach_slot_transport",
           [](BandPipeline& p, int k, std::shared_ptr<HaloTransport> t) { p.set_slot_transport(k, std::move(t)); },
           py::keep_alive<1, 3>())
      .def(
          "submit",
          [](BandPipeline& p, uintptr_t in_ptr, int64_t in_r0, int64_t in_r1, uintptr_t out_ptr, int reps) {
            py::gil_scoped_release nogil;
            p.submit(reinterpret_cast<const uint8_t*>(in_ptr), in_r0, in_r1, reinterpret_cast<uint8_t*>(out_ptr), reps);
          },
          py::arg("in_ptr"), py::arg("in_r0"), py::arg("in_r1"), py::arg("out_ptr"), py::arg("reps"))
      .def("drain", &BandPipeline::drain, py::call_guard<py::gil_scoped_release>())
      .def("ready", &BandPipeline::ready, py::arg("slot"), "slot-stream mode: the slot's latest image is done")
      .def("wait_image", &BandPipeline::wait_image, py::arg("slot"), py::call_guard<py::gil_scoped_release>(),
           "slot-stream mode: block until the slot's latest image is done")
      .def("enable_marks", &BandPipeline::enable_marks, py::arg("images"),
           "Completion marks of the next `images` submits (a diagnostic pass; see marks()).")
      .def("marks", &BandPipeline::marks, py::call_guard<py::gil_scoped_release>(),
           "Drain, then per marked image [slot, ms from the first image's issue to its completion, head-streamed].")
      .def_property_readonly("submitted", &BandPipeline::submitted)
      .def_property_readonly("concurrent", &BandPipeline::concurrent)
      .def_property_readonly("graphs", &BandPipeline::graphs)
      .def_property_readonly("streamed_heads", &BandPipeline::streamed_heads)
      .def_property_readonly("step_graphs", &BandPipeline::step_graphs)
      .def_property_readonly("options",
                             [](BandPipeline& p) {
                               const EngineOptions& o = p.slot(0).options();
                               py::dict d;
                               d["stream_chunks"] = o.stream_chunks;
                               d["stream_weights"] = o.stream_weights;
                               d["lazy_head"] = o.lazy_head;
                               d["stream_min_bytes"] = o.stream_min_bytes;
                               d["head_alt_uploads"] = o.head_alt_uploads;
                               d["cu_mask_queues"] = o.cu_mask_queues;
                               d["head_on_slot_streams"] = o.head_on_slot_streams;
                               return d;
                             })
      .def("enable_trace", &BandPipeline::enable_trace, py::arg("images"),
           "Time the stages of the next `images` submits (directly issued pipelines only)")
      .def("trace", &BandPipeline::trace, py::call_guard<py::gil_scoped_release>(),
           "Per traced image: [slot, H2D start, H2D end, reps end, D2H end] in ms");

  py::class_<LocalCluster>(m, "LocalCluster")
      .def(py::init([](int64_t w, int64_t h, const std::string& ch, py::object filter, int bands, int device, int halo,
                       int fuse, const std::string& variant, bool overlap) {
             EngineOptions o;
             o.device = device;
             o.halo_depth = halo;
             o.fuse = fuse;
             o.overlap = overlap;
             o.variant = parse_variant(variant);
             return std::make_unique<LocalCluster>(make_geom(w, h, ch), bands, make_filter(filter), o);
           }),
           py::arg("width"), py::arg("height"), py::arg("channels"), py::arg("filter") = "gaussian",
           py::arg("bands") = 2, py::arg("device") = 0, py::arg("halo") = 1, py::arg("fuse") = 1,
           py::arg("variant") = "auto", py::arg("overlap") = true)
      .def("upload",
           [](LocalCluster& c, py::buffer host, bool preload_halo) {
             c.upload(host_view(host, false).ptr, preload_halo);
           },
           py::arg("host"), py::arg("preload_halo") = false)
      .def("run", &LocalCluster::run, py::arg("reps"), py::arg("device_async") = false,
           py::call_guard<py::gil_scoped_release>(),
           "device_async: every band through the production phase path (comm stream || interior, event-ordered)")
      .def("download", [](LocalCluster& c, py::buffer host) { c.download(host_view(host, true).ptr); })
      .def("exchanges", [](LocalCluster& c) { return c.engine(0).last_stats().exchanges; })
      .def_property_readonly("size", &LocalCluster::size);

  // ---------------------------------------------------------------- HIP IPC halos
  m.def("ipc_create_segment", &ipc_create_segment, py::arg("name"), py::arg("world"), py::arg("slots"),
        "create the zeroed shared flag segment of an IPC halo job (one rank)");
  m.def("ipc_pull_probe", &ipc_pull_probe, py::arg("form"), py::arg("bytes"), py::arg("host_source"),
        py::arg("iters") = 50, py::arg("device") = 0, py::arg("workgroups") = 0,
        py::call_guard<py::gil_scoped_release>(),
        "ms per IPC exchange of one pull form (grid|single|sdma), `bytes` per side from a pinned host buffer "
        "(host_source: stand-in for a peer GPU behind xGMI) or this GPU's HBM; self-neighbour flag protocol");
  m.def("ipc_grid_workgroups", &ipc_grid_workgroups, py::arg("bytes"));
  m.def("ipc_unlink_segment", &ipc_unlink_segment, py::arg("name"),
        "remove the segment's name (mappings stay valid; call once every rank has mapped it)");
  py::class_<IpcHaloTransport, HaloTransport, std::shared_ptr<IpcHaloTransport>>(m, "IpcHaloTransport")
      .def(py::init([](BandEngine& e, const std::string& segment, int slot, int slots, double timeout_s,
                       const std::string& pull) {
             return std::make_shared<IpcHaloTransport>(e, segment, slot, slots, timeout_s, parse_ipc_pull(pull));
           }),
           py::arg("engine"), py::arg("segment"), py::arg("slot") = 0, py::arg("slots") = 1,
           py::arg("timeout_s") = 30.0, py::arg("pull") = "grid", py::keep_alive<1, 2>())
      .def_property_readonly("pull", [](const IpcHaloTransport& t) { return std::string(ipc_pull_name(t.pull())); })
      .def("local_handles", [](const IpcHaloTransport& t) {
        const auto v = t.local_handles();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("connect",
           [](IpcHaloTransport& t, py::bytes up, py::bytes down) {
             const std::string u = up, d = down;
             t.connect(std::vector<uint8_t>(u.begin(), u.end()), std::vector<uint8_t>(d.begin(), d.end()));
           },
           py::arg("up"), py::arg("down"))
      .def_property_readonly("connected", &IpcHaloTransport::connected)
      .def("self_test", &IpcHaloTransport::self_test, py::arg("timeout_s") = 5.0,
           py::call_guard<py::gil_scoped_release>(),
           "collective: one exchange of sentinel rows with the neighbours, compared; raises a named error")
      .def_property_readonly("self_tested", &IpcHaloTransport::self_tested)
      .def_property_readonly("mailbox_kind", &IpcHaloTransport::mailbox_kind)
      .def("peer_device", &IpcHaloTransport::peer_device, py::arg("side"))
      .def_property_readonly("enqueued", &IpcHaloTransport::enqueued)
      .def_property_readonly("device_count", &IpcHaloTransport::device_count)
      .def("check", &IpcHaloTransport::check, "raise if a wait of this rank timed out (after the stream drained)");

  // ---------------------------------------------------------------- RCCL
  m.def("rccl_unique_id", []() {
    const auto v = rccl_unique_id();
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
  });
  m.def("rccl_version", &rccl_version);
  m.def("rccl_loaded", &rccl_loaded, "True once librccl is mapped (loaded lazily on the first RCCL call)");
  m.def("install_crash_handler", &install_crash_handler,
        "print a native backtrace on SIGSEGV/SIGBUS/SIGILL/SIGFPE/SIGABRT, then chain to the previous handler");
  m.def("rccl_capture_probe", &rccl_capture_probe, py::arg("op") = "sendrecv", py::arg("mode") = "relaxed",
        py::arg("bytes") = 4096, py::arg("device") = 0, py::arg("launches") = 3,
        py::call_guard<py::gil_scoped_release>());
  m.def("rccl_selftest_exchange", &rccl_selftest_exchange, py::arg("device") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("rccl_selftest_multicomm", &rccl_selftest_multicomm, py::arg("device") = 0, py::arg("slots") = 3,
        py::arg("images") = 60, py::arg("timeout_s") = 60.0, py::call_guard<py::gil_scoped_release>());
  m.def("rccl_library_path", &rccl_library_path, "path of the mapped librccl ('' while none is mapped)");
  m.def(
      "runtime_info",
      []() {
        const HipRuntimeInfo h = hip_runtime_info();
        py::dict d;
        d["hip_runtime_version"] = h.runtime_version;
        d["hip_driver_version"] = h.driver_version;
        d["hip_runtime_path"] = h.runtime_path;
        d["hip_compiled_version"] = h.compiled_version;
        const bool loaded = rccl_loaded();
        d["rccl_version"] = loaded ? py::object(py::str(rccl_version())) : py::object(py::none());
        d["rccl_path"] = loaded ? py::object(py::str(rccl_library_path())) : py::object(py::none());
        return d;
      },
      "the HIP runtime / RCCL this process actually runs on (versions and library paths)");
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](py::bytes id, int rank, int world, int device) {
             const std::string s = id;
             std::vector<uint8_t> v(s.begin(), s.end());
             py::gil_scoped_release nogil;
             return std::make_shared<RcclComm>(v, rank, world, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def("allreduce_max", &RcclComm::allreduce_max, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_sum", &RcclComm::allreduce_sum, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &RcclComm::barrier, py::call_guard<py::gil_scoped_release>())
      .def(
          "wait",
          [](RcclComm& c, uintptr_t stream, double timeout_s) { c.wait(reinterpret_cast<hipStream_t>(stream), timeout_s); },
          py::arg("stream"), py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>(),
          "Wait for a stream while polling RCCL async errors; aborts the communicator and raises on timeout.");

  m.def("set_error_rank", &set_error_rank);
}

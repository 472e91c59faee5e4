// Band schedule planner (see schedule.hpp).
#include "pconv/schedule.hpp"

#include <algorithm>
#include <sstream>

#include "pconv/common.hpp"

namespace pconv {

PlanConfig normalize_plan_config(PlanConfig cfg, int64_t min_band_rows, int max_fuse) {
  cfg.fuse = std::max(1, std::min(cfg.fuse, max_fuse));
  cfg.halo_depth = std::max(cfg.halo_depth, cfg.fuse);
  // Ghost rows of a band come from the adjacent band only.
  if (min_band_rows > 0 && cfg.halo_depth > min_band_rows)
    cfg.halo_depth = static_cast<int>(std::max<int64_t>(1, min_band_rows));
  cfg.fuse = std::min(cfg.fuse, cfg.halo_depth);
  return cfg;
}

std::vector<Phase> plan_band(const Band& band, int reps, const PlanConfig& cfg) {
  PCONV_CHECK(reps >= 0, "reps must be >= 0");
  PCONV_CHECK(cfg.fuse >= 1 && cfg.halo_depth >= cfg.fuse, "plan: need 1 <= fuse <= halo_depth");
  const bool has_up = band.up >= 0, has_down = band.down >= 0;
  const bool has_nb = has_up || has_down;
  const int64_t rows = band.rows;
  PCONV_CHECK(!has_nb || cfg.halo_depth <= rows, "plan: halo depth exceeds band rows");

  std::vector<Phase> plan;
  int64_t ghost = cfg.halo_preloaded ? cfg.halo_depth : 0;  // valid ghost rows in src
  int done = 0;
  while (done < reps) {
    Phase ph;
    const int s = std::min(cfg.fuse, reps - done);
    ph.steps = s;
    if (has_nb && ghost < s) {
      ph.exchange_depth = cfg.halo_depth;
      ghost = cfg.halo_depth;
    }
    const int64_t ext = has_nb ? ghost - s : 0;
    const int64_t lo = has_up ? -ext : 0;
    const int64_t hi = has_down ? rows + ext : rows;
    if (ph.exchange_depth > 0 && cfg.overlap) {
      // Interior: outputs whose s-step dependency cone stays inside owned
      // rows (or inside the zero rows beyond a global image edge).
      const int64_t ilo = has_up ? s : 0;
      const int64_t ihi = has_down ? rows - s : rows;
      if (ihi > ilo) {
        ph.launches.push_back({s, ilo, ihi, false});
        if (lo < ilo) ph.launches.push_back({s, lo, ilo, true});
        if (ihi < hi) ph.launches.push_back({s, ihi, hi, true});
      } else {
        ph.launches.push_back({s, lo, hi, true});
      }
    } else {
      ph.launches.push_back({s, lo, hi, ph.exchange_depth > 0});
    }
    if (has_nb) ghost -= s;
    done += s;
    plan.push_back(std::move(ph));
  }
  return plan;
}

bool streamable(const std::vector<Phase>& plan) {
  if (plan.empty()) return false;
  for (const auto& p : plan)
    if (p.exchange_depth > 0 || p.launches.size() != 1) return false;
  return true;
}

std::vector<int64_t> stream_cuts(int64_t in_lo, int64_t in_hi, int chunks) {
  const int64_t n = in_hi - in_lo;
  chunks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(chunks, n)));
  if (chunks <= 1) return {};
  std::vector<int> w(static_cast<size_t>(chunks), 5);  // 5, ..., 5, 6
  w.back() = 6;
  return stream_cuts_weighted(in_lo, in_hi, w);
}

std::vector<int64_t> stream_cuts_weighted(int64_t in_lo, int64_t in_hi, const std::vector<int>& weights) {
  const int64_t n = in_hi - in_lo;
  int64_t total = 0;
  for (int w : weights) {
    PCONV_CHECK(w > 0, "stream_cuts_weighted: weights must be positive");
    total += w;
  }
  std::vector<int64_t> cuts;
  int64_t acc = 0;
  for (size_t c = 0; c + 1 < weights.size(); ++c) {
    acc += weights[c];
    const int64_t cut = in_lo + (n * acc) / total;
    if (cut > in_lo && cut < in_hi && (cuts.empty() || cut > cuts.back())) cuts.push_back(cut);
  }
  return cuts;
}

StreamPlan plan_streamed(const std::vector<Phase>& plan, int64_t in_lo, int64_t in_hi, int64_t owned_rows,
                         const std::vector<int64_t>& cuts) {
  PCONV_CHECK(streamable(plan), "plan_streamed: the plan must be exchange-free with one launch per phase");
  PCONV_CHECK(in_lo <= 0 && in_hi >= owned_rows && in_lo < in_hi, "plan_streamed: input rows must cover the band");
  for (size_t i = 0; i < cuts.size(); ++i)
    PCONV_CHECK(cuts[i] > in_lo && cuts[i] < in_hi && (i == 0 || cuts[i] > cuts[i - 1]),
                "plan_streamed: cuts must increase strictly inside the input rows");
  const int L = static_cast<int>(plan.size());
  std::vector<int64_t> lo(L + 1), hi(L + 1);
  std::vector<int> s(L + 1, 0);
  lo[0] = in_lo;
  hi[0] = in_hi;
  for (int j = 1; j <= L; ++j) {
    const LaunchSpec& l = plan[j - 1].launches[0];
    lo[j] = l.lo;
    hi[j] = l.hi;
    s[j] = l.steps;
  }
  PCONV_CHECK(lo[L] <= 0 && hi[L] >= owned_rows, "plan_streamed: the last level must cover the owned rows");
  StreamPlan sp;
  sp.levels = L;
  std::vector<int64_t> front(lo);  // W_j(c-1): first row of level j not yet computed
  front[0] = in_lo;
  const size_t C = cuts.size() + 1;
  for (size_t c = 0; c < C; ++c) {
    const bool last = c + 1 == C;
    StreamChunk ch;
    ch.up_lo = front[0];
    ch.up_hi = last ? in_hi : cuts[c];
    std::vector<int64_t> w(L + 1);
    w[0] = ch.up_hi;
    for (int j = 1; j <= L; ++j) {
      int64_t wj;
      if (last || w[j - 1] >= hi[j - 1])
        wj = hi[j];
      else
        wj = std::min(hi[j], w[j - 1] - std::max(s[j], s[j - 1]));
      wj = std::max(wj, front[j]);
      w[j] = wj;
      if (wj > front[j]) {
        ch.launches.push_back({s[j], front[j], wj, false});
        ch.levels.push_back(j);
      }
    }
    ch.down_lo = std::max<int64_t>(0, front[L]);
    ch.down_hi = std::min(owned_rows, w[L]);
    if (ch.down_hi < ch.down_lo) ch.down_hi = ch.down_lo;
    for (int j = 0; j <= L; ++j) front[j] = w[j];
    sp.chunks.push_back(std::move(ch));
  }
  return sp;
}

std::string describe_plan(const std::vector<Phase>& plan) {
  std::ostringstream os;
  for (size_t i = 0; i < plan.size(); ++i) {
    const Phase& p = plan[i];
    os << "phase " << i << ": steps=" << p.steps;
    if (p.exchange_depth) os << " exchange=" << p.exchange_depth;
    for (const auto& l : p.launches)
      os << " [" << l.lo << "," << l.hi << ")" << (l.after_halo ? "*" : "");
    os << "\n";
  }
  return os.str();
}

}  // namespace pconv

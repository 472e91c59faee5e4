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

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
  std::vector<int64_t> cuts;
  if (chunks <= 1) return cuts;
  // weights 1, 2, ..., 2, 1 (two chunks: 1, 1)
  const int64_t total = chunks == 2 ? 2 : 2 * (chunks - 1);
  int64_t acc = 0;
  for (int c = 0; c + 1 < chunks; ++c) {
    acc += (c == 0 || chunks == 2) ? 1 : 2;
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

namespace {

int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

}  // namespace

WavePlan plan_wave(const std::vector<Phase>& plan, int64_t in_lo, int64_t in_hi, int64_t owned_rows, int tile_rows,
                   const std::vector<int>& col_groups, int load_parts, int store_parts, int load_lead,
                   int level_gap) {
  PCONV_CHECK(streamable(plan), "plan_wave: the plan must be exchange-free with one launch per phase");
  PCONV_CHECK(in_lo <= 0 && in_hi >= owned_rows && in_lo < in_hi, "plan_wave: input rows must cover the band");
  PCONV_CHECK(tile_rows >= 1 && load_parts >= 1 && store_parts >= 1, "plan_wave: bad tiling");
  const int L = static_cast<int>(plan.size());
  PCONV_CHECK(static_cast<int>(col_groups.size()) >= L + 1, "plan_wave: one column-group count per level");
  WavePlan wp;
  wp.levels = L;
  wp.tile_rows = tile_rows;
  wp.steps.assign(L + 1, 0);
  wp.lo.assign(L + 1, in_lo);
  wp.hi.assign(L + 1, in_hi);
  for (int j = 1; j <= L; ++j) {
    const LaunchSpec& l = plan[j - 1].launches[0];
    wp.steps[j] = l.steps;
    wp.lo[j] = l.lo;
    wp.hi[j] = l.hi;
    PCONV_CHECK(l.hi > l.lo && col_groups[j] >= 1, "plan_wave: empty level");
  }
  PCONV_CHECK(wp.lo[L] <= 0 && wp.hi[L] >= owned_rows, "plan_wave: the last level must cover the owned rows");
  const int64_t V = tile_rows;
  wp.tiles.resize(L + 1);
  wp.arrivals.resize(L + 1);
  wp.counter_base.resize(L + 1);
  for (int j = 0; j <= L; ++j) {
    wp.tiles[j] = static_cast<int>((wp.hi[j] - wp.lo[j] + V - 1) / V);
    wp.arrivals[j] = j == 0 ? load_parts : col_groups[j];
    wp.counter_base[j] = wp.counters;
    wp.counters += wp.tiles[j];
  }
  auto tile_a = [&](int j, int64_t t) { return wp.lo[j] + t * V; };
  auto tile_b = [&](int j, int64_t t) { return std::min(wp.lo[j] + (t + 1) * V, wp.hi[j]); };
  // Tiles of level j overlapping rows [r0, r1) (clipped to the level).
  auto tiles_of = [&](int j, int64_t r0, int64_t r1, int64_t& t0, int64_t& t1) {
    r0 = std::max(r0, wp.lo[j]);
    r1 = std::min(r1, wp.hi[j]);
    if (r1 <= r0) {
      t0 = 0;
      t1 = -1;
      return;
    }
    t0 = floor_div(r0 - wp.lo[j], V);
    t1 = floor_div(r1 - 1 - wp.lo[j], V);
  };
  struct Keyed {
    int64_t rank;
    WaveTask t;
  };
  std::vector<Keyed> all;
  std::vector<std::vector<int64_t>> rank(L + 1);
  const int64_t kLoadLead = std::max(0, load_lead);  // loads take their tickets this many ranks early
  // rows of a tile split into `parts` row parts (empty parts dropped)
  auto parts_of = [](int64_t a, int64_t b, int parts, int p, int64_t& pa, int64_t& pb) {
    pa = a + (b - a) * p / parts;
    pb = a + (b - a) * (p + 1) / parts;
  };
  // level 0: loads
  rank[0].assign(wp.tiles[0], 0);
  for (int64_t t = 0; t < wp.tiles[0]; ++t) {
    rank[0][t] = t;
    for (int p = 0; p < load_parts; ++p) {
      WaveTask k;
      int64_t pa, pb;
      parts_of(tile_a(0, t), tile_b(0, t), load_parts, p, pa, pb);
      k.kind = 0;
      k.level = 0;
      k.a = static_cast<int32_t>(pa);
      k.b = static_cast<int32_t>(pb);
      k.part = p;
      k.tile = static_cast<int32_t>(t);
      all.push_back({t - kLoadLead, k});
    }
  }
  for (int j = 1; j <= L; ++j) {
    rank[j].assign(wp.tiles[j], 0);
    const int64_t s = wp.steps[j], sp = wp.steps[j - 1];
    for (int64_t t = 0; t < wp.tiles[j]; ++t) {
      const int64_t a = tile_a(j, t), b = tile_b(j, t);
      int64_t r0, r1;
      tiles_of(j - 1, a - s, b + s, r0, r1);  // rows it reads
      PCONV_CHECK(r1 >= r0, "plan_wave: a level tile reads nothing of the level before");
      if (j >= 2) {
        // level-(j-1) tiles whose reads [a'-sp, b'+sp) reach rows [a, b) of
        // level j-2, which this tile overwrites
        int64_t w0, w1;
        tiles_of(j - 1, a - sp, b + sp, w0, w1);
        if (w1 >= w0) {
          r0 = std::min(r0, w0);
          r1 = std::max(r1, w1);
        }
      }
      r0 = std::max<int64_t>(r0, 0);
      r1 = std::min<int64_t>(r1, wp.tiles[j - 1] - 1);
      int64_t rk = 0;
      for (int64_t d = r0; d <= r1; ++d) rk = std::max(rk, rank[j - 1][d]);
      rank[j][t] = rk + std::max(1, level_gap);
      for (int g = 0; g < col_groups[j]; ++g) {
        WaveTask k;
        k.kind = 1;
        k.level = j;
        k.a = static_cast<int32_t>(a);
        k.b = static_cast<int32_t>(b);
        k.part = g;
        k.tile = static_cast<int32_t>(t);
        k.dep_lo = static_cast<int32_t>(r0);
        k.dep_hi = static_cast<int32_t>(r1);
        all.push_back({rank[j][t], k});
      }
    }
  }
  // stores: the owned rows of each level-L tile
  for (int64_t t = 0; t < wp.tiles[L]; ++t) {
    const int64_t a = std::max<int64_t>(tile_a(L, t), 0), b = std::min<int64_t>(tile_b(L, t), owned_rows);
    if (b <= a) continue;
    for (int p = 0; p < store_parts; ++p) {
      WaveTask k;
      int64_t pa, pb;
      parts_of(a, b, store_parts, p, pa, pb);
      if (pb <= pa) continue;
      k.kind = 2;
      k.level = L + 1;
      k.a = static_cast<int32_t>(pa);
      k.b = static_cast<int32_t>(pb);
      k.part = p;
      k.tile = static_cast<int32_t>(t);
      k.dep_lo = k.dep_hi = static_cast<int32_t>(t);
      all.push_back({rank[L][t] + 1, k});
    }
  }
  std::stable_sort(all.begin(), all.end(), [](const Keyed& x, const Keyed& y) {
    return x.rank != y.rank ? x.rank < y.rank : x.t.level < y.t.level;
  });
  wp.tasks.reserve(all.size());
  for (const auto& k : all) wp.tasks.push_back(k.t);
  check_wave_order(wp);
  return wp;
}

void check_wave_order(const WavePlan& wp) {
  // arrivals seen so far per counter, in ticket order
  std::vector<int> seen(static_cast<size_t>(wp.counters), 0);
  for (size_t i = 0; i < wp.tasks.size(); ++i) {
    const WaveTask& k = wp.tasks[i];
    const int dl = k.dep_level();
    if (dl >= 0) {
      PCONV_CHECK(dl <= wp.levels && k.dep_lo <= k.dep_hi, "wave plan: dependency out of range");
      for (int d = k.dep_lo; d <= k.dep_hi; ++d) {
        PCONV_CHECK(d >= 0 && d < wp.tiles[dl], "wave plan: dependency tile out of range");
        PCONV_CHECK(seen[wp.counter_base[dl] + d] == wp.arrivals[dl],
                    "wave plan: task " + std::to_string(i) + " waits on a tile whose tasks are not all earlier");
      }
    }
    if (k.kind != 2) ++seen[wp.counter_base[k.level] + k.tile];
  }
  for (int j = 0; j <= wp.levels; ++j)
    for (int t = 0; t < wp.tiles[j]; ++t)
      PCONV_CHECK(seen[wp.counter_base[j] + t] == wp.arrivals[j], "wave plan: a tile misses tasks");
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

// Host-side check of the weight-gradient schedules (csrc/wgrad.hpp WgPlan, run by tests/test_wgrad_plan.py;
// no GPU call). For the problem list train.hip's uavhip_ppo_step builds at minibatch Bm, and for both
// schedules (stream-K and chunked), it replays k_wgrad's per-workgroup decode on the host and checks:
//   * every (problem, tile, k-slab) unit is computed by exactly one run;
//   * every run writes its own partial slot, inside the kWgGrid x kWgRuns slot buffer;
//   * the reduction map (WgPlan::tiles: first slot, second slot, then every run_stride slots) names
//     exactly the slots of that tile's runs.
// Prints one line per case and exits non-zero on the first violation.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#include "common.hpp"
#include "wgrad.hpp"

using namespace uavhip::tr;

namespace {
constexpr int D = 128, FF = 256, HID = 64, S = 5;
alignas(16) float g_dummy[64];

// train.hip layer_dw: C0 (full, R rows: Q, K, V rows as three problems), A and C1 (pruned: K and V
// over R rows, the rest over Bm), the heads; the key-row problems three-plane (p3_tiles)
bool build(WgPlan& wp, int Bm) {
    const int R = S * Bm;
    auto dw = [&](int M, int N, int K, int p3 = 0) {
        wp.add(g_dummy, M, g_dummy, N, M, N, K);
        if (wp.ok) wp.b.p[wp.b.n - 1].p3_tiles = p3;
    };
    dw(D, D, R);
    dw(D, D, R, 1);
    dw(D, D, R);
    dw(D, D, R);
    dw(FF, D, R);
    dw(D, FF, R);
    for (int l = 0; l < 2; ++l) {
        dw(D, D, R, 1);
        dw(D, D, R);
        dw(D, D, Bm);
        dw(D, D, Bm);
        dw(FF, D, Bm);
        dw(D, FF, Bm);
    }
    dw(HID, D, Bm);
    dw(HID, D, Bm);
    return wp.ok;
}

int fail(const char* what, int Bm, const char* mode) {
    std::printf("FAIL Bm=%d %s: %s\n", Bm, mode, what);
    return 1;
}

// k_wgrad's decode for workgroup b of the launch (wgrad.hpp), as host code
struct Run {
    int prob, tile, s0, n, slot;
};
std::vector<Run> decode(const WgBatch& wb, int G, int b) {
    std::vector<Run> runs;
    long long U = wb.units;
    int u = (int)(b * U / G), u_end = (int)((b + 1) * U / G), slot_wg = b;
    if (wb.chunk) {
        slot_wg = (b & 7) * (G >> 3) + (b >> 3);
        if (slot_wg >= wb.wgs) return runs;
        int qi = 0;
        while (qi + 1 < wb.n && slot_wg >= wb.p[qi + 1].wg_begin) ++qi;
        const WgProb& Q = wb.p[qi];
        const int local = slot_wg - Q.wg_begin, c = local / Q.tiles, t = local - c * Q.tiles;
        const int s0 = c * Q.chunk;
        u = Q.unit_begin + t * Q.slabs + s0;
        u_end = u + std::min(Q.chunk, Q.slabs - s0);
    }
    int run = 0;
    while (u < u_end) {
        int pi = 0;
        while (pi + 1 < wb.n && u >= wb.p[pi + 1].unit_begin) ++pi;
        const WgProb& P = wb.p[pi];
        const int local = u - P.unit_begin, tile = local / P.slabs, s0 = local - tile * P.slabs;
        const int n = std::min(u_end - u, P.slabs - s0);
        runs.push_back(Run{pi, tile, s0, n, slot_wg * kWgRuns + run});
        u += n;
        ++run;
    }
    return runs;
}

int check(int Bm, bool chunked) {
    const char* mode = chunked ? "chunked" : "stream-K";
    WgPlan wp;
    if (!build(wp, Bm)) return fail("problem list rejected", Bm, mode);
    if (chunked && !wp.chunked()) return fail("no chunk size fits the grid", Bm, mode);
    std::vector<WgTileRuns> segs;
    if (!wp.tiles([&](const WgTileRuns& t) { segs.push_back(t); })) return fail("tiles() refused", Bm, mode);
    const WgBatch& wb = wp.b;
    const int G = wp.grid;
    if (G <= 0 || G > kWgGrid) return fail("grid out of range", Bm, mode);
    if (chunked && G % 8) return fail("chunked grid not a multiple of 8", Bm, mode);
    std::map<long long, int> cover;             // (prob, tile, slab) -> count
    std::map<std::pair<int, int>, std::set<int>> slots_of;  // (prob, tile) -> slots written
    std::set<int> slots;
    for (int b = 0; b < G; ++b) {
        const std::vector<Run> rs = decode(wb, G, b);
        if ((int)rs.size() > kWgRuns) return fail("more runs than slots in a workgroup", Bm, mode);
        for (const Run& r : rs) {
            if (r.slot < 0 || r.slot >= kWgGrid * kWgRuns) return fail("slot outside the buffer", Bm, mode);
            if (!slots.insert(r.slot).second) return fail("two runs share a slot", Bm, mode);
            slots_of[{r.prob, r.tile}].insert(r.slot);
            for (int s = r.s0; s < r.s0 + r.n; ++s) ++cover[((long long)r.prob * 64 + r.tile) * 100000 + s];
        }
    }
    long long units = 0;
    for (int pi = 0; pi < wb.n; ++pi) {
        const WgProb& P = wb.p[pi];
        for (int t = 0; t < P.tiles; ++t)
            for (int s = 0; s < P.slabs; ++s) {
                ++units;
                auto it = cover.find(((long long)pi * 64 + t) * 100000 + s);
                if (it == cover.end() || it->second != 1) return fail("a unit not computed exactly once", Bm, mode);
            }
    }
    if ((long long)cover.size() != units) return fail("units outside the problems", Bm, mode);
    if ((int)segs.size() != wb.tiles) return fail("reduction map: one entry per tile", Bm, mode);
    for (const WgTileRuns& t : segs) {
        const WgProb& P = wb.p[t.prob];
        const int tile = (t.m0 / kWgT) * P.tiles_n + t.n0 / kWgT;
        std::set<int> named;
        named.insert(t.first_slot);
        for (int r = 1; r < t.runs; ++r) named.insert(t.rest_slot + (r - 1) * t.run_stride);
        if ((int)named.size() != t.runs) return fail("reduction map names a slot twice", Bm, mode);
        if (named != slots_of[{t.prob, tile}]) return fail("reduction map != the tile's run slots", Bm, mode);
        if (t.rows != std::min(kWgT, P.M - t.m0)) return fail("tile rows", Bm, mode);
    }
    int ch3 = 0;
    for (int pi = 0; pi < wb.n; ++pi)
        if (wb.p[pi].p3_tiles) ch3 = wb.p[pi].chunk;
    std::printf("ok Bm=%d %s: %d problems, %d tiles, %lld units, grid %d, chunk %d (three-plane %d)\n", Bm, mode,
                wb.n, wb.tiles, units, G, wb.chunk, ch3);
    return 0;
}
}  // namespace

int main(int argc, char** argv) {
    int rc = 0;
    for (int i = 1; i < argc; ++i) {
        const int Bm = std::atoi(argv[i]);
        rc |= check(Bm, false);
        rc |= check(Bm, true);
    }
    return rc;
}

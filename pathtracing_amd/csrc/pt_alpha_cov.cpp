// Conservative alpha coverage masks (pt_alpha_cov.h).  Host code.
#include "pt_alpha_cov.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace {
constexpr uint32_t SRC_CH4 = 0, SRC_CH1 = 1, SRC_CONST = 2;  // pt_device.h ALPHA_SRC_*
constexpr uint32_t M_OPAQUE = 0, M_BLEND = 1, M_MASK = 2;    // pt_api.h PT_ALPHA_*
constexpr uint32_t ALL = 0xFFFFu;
// texel-space footprints beyond this are left to the exact test (floor and
// the int conversion of such coordinates are not worth reasoning about)
constexpr double MAX_COORD = 16777216.0;
// images above this many texels get no square tables (memory: 2 bytes per
// texel per level); their cells stay undecided
constexpr uint64_t MAX_PYRAMID_TEXELS = 1ull << 24;
constexpr int MAX_LEVEL = 6;  // squares up to 64 x 64

// the decision for a value range [lo, hi] of the alpha a, as the reference's
// AlphaTester (Material.hpp:184-195) and tri_alpha_rec (pt_trace.h) decide it:
// 1 accept, 2 reject, 0 undecided
int decide(uint32_t mode, double lo, double hi, float cut) {
    if (mode == M_OPAQUE) return 1;
    if (!(lo <= hi)) return 0;  // NaN
    if (mode == M_MASK) {       // a > cutoff
        if (lo > (double)cut) return 1;
        if (hi <= (double)cut) return 2;
        return 0;
    }
    // BLEND: a >= 1 ? true : random_float() < a, random in [0, 1)
    if (lo >= 1.0) return 1;
    if (hi <= 0.0) return 2;
    return 0;
}

// the column (or row) ranges of a footprint [X0, X1] of unwrapped texel
// coordinates on an axis of n texels (repeat wrap, Texture.hpp GetChannelAt):
// one or two in-image ranges
int wrap_ranges(int64_t X0, int64_t X1, int n, int r[2][2]) {
    if (X1 - X0 + 1 >= n) {
        r[0][0] = 0, r[0][1] = n - 1;
        return 1;
    }
    int64_t a = X0 % n;
    if (a < 0) a += n;
    const int64_t b = a + (X1 - X0);
    if (b < n) {
        r[0][0] = (int)a, r[0][1] = (int)b;
        return 1;
    }
    r[0][0] = (int)a, r[0][1] = n - 1;
    r[1][0] = 0, r[1][1] = (int)(b - n);
    return 2;
}
}  // namespace

uint64_t PtAlphaCoverage::Pyramid::query(int x0, int x1, int y0, int y1, uint8_t& lo, uint8_t& hi) const {
    const int w = x1 - x0 + 1, h = y1 - y0 + 1;
    int k = 0;
    while (k + 1 < (int)mn.size() && (2 << k) <= std::min(w, h)) k++;
    const int s = 1 << k;
    const std::vector<uint8_t>& A = mn[k];
    const std::vector<uint8_t>& B = mx[k];
    uint64_t n = 0;
    for (int y = y0;; y += s) {
        const int yy = std::min(y, y1 - s + 1);
        for (int x = x0;; x += s) {
            const size_t i = (size_t)yy * W + std::min(x, x1 - s + 1);
            lo = std::min(lo, A[i]);
            hi = std::max(hi, B[i]);
            n++;
            if (x + s > x1) break;
        }
        if (y + s > y1) break;
    }
    return n;
}

const PtAlphaCoverage::Pyramid* PtAlphaCoverage::pyramid(uint64_t off, uint32_t W, uint32_t H, uint32_t C,
                                                         uint32_t ch) {
    const auto key = std::make_tuple(off, W, H, C, ch);
    auto it = pyr_.find(key);
    if (it != pyr_.end()) return it->second.get();
    std::unique_ptr<Pyramid> p;
    const uint64_t bytes = (uint64_t)W * H * C;
    if (W && H && ch < C && (uint64_t)W * H <= MAX_PYRAMID_TEXELS && off <= n_ && bytes <= n_ - off) {
        p = std::make_unique<Pyramid>();
        p->W = (int)W, p->H = (int)H;
        const size_t n = (size_t)W * H;
        p->mn.emplace_back(n), p->mx.emplace_back(n);
        const uint8_t* base = texels_ + off;
        for (size_t k = 0; k < n; k++) p->mn[0][k] = p->mx[0][k] = base[k * C + ch];
        for (int k = 1; k <= MAX_LEVEL && (1u << k) <= std::min(W, H); k++) {
            const int hs = 1 << (k - 1), lim_x = (int)W - (1 << k), lim_y = (int)H - (1 << k);
            std::vector<uint8_t> mn(n, 255), mx(n, 0);
            const auto& pmn = p->mn.back();
            const auto& pmx = p->mx.back();
            for (int y = 0; y <= lim_y; y++)
                for (int x = 0; x <= lim_x; x++) {
                    const size_t i = (size_t)y * W + x, r = i + hs, d = i + (size_t)hs * W, e = d + hs;
                    mn[i] = std::min(std::min(pmn[i], pmn[r]), std::min(pmn[d], pmn[e]));
                    mx[i] = std::max(std::max(pmx[i], pmx[r]), std::max(pmx[d], pmx[e]));
                }
            p->mn.push_back(std::move(mn)), p->mx.push_back(std::move(mx));
        }
    }
    return (pyr_[key] = std::move(p)).get();
}

// min / max byte of every texel a bilinear lookup at a point of the texel-
// space triangle (px, py), widened by (mx, my), can read.  The triangle is
// walked in bands of rows; each band's rectangle spans the triangle's x-extent
// over the band (widened), so the footprint follows the triangle's shape, not
// its bounding box.  False when the coordinates are too large to reason about.
bool PtAlphaCoverage::footprint(const Pyramid& P, const double px[3], const double py[3], double mx, double my,
                                uint8_t& blo, uint8_t& bhi) {
    double ylo = std::min({py[0], py[1], py[2]}) - my, yhi = std::max({py[0], py[1], py[2]}) + my;
    double xlo = std::min({px[0], px[1], px[2]}) - mx, xhi = std::max({px[0], px[1], px[2]}) + mx;
    if (!(std::fabs(ylo) < MAX_COORD && std::fabs(yhi) < MAX_COORD && std::fabs(xlo) < MAX_COORD &&
          std::fabs(xhi) < MAX_COORD))
        return false;
    // a footprint spanning a whole axis of the image: its bounding rectangle
    // (every row or every column, wrapped) -- conservative, and bounded work
    // for triangles whose uvs tile the image many times
    if (yhi - ylo + 2.0 >= (double)P.H || xhi - xlo + 2.0 >= (double)P.W) {
        int rx[2][2], ry[2][2];
        const int nx = wrap_ranges((int64_t)std::floor(xlo), (int64_t)std::floor(xhi) + 1, P.W, rx);
        const int ny = wrap_ranges((int64_t)std::floor(ylo), (int64_t)std::floor(yhi) + 1, P.H, ry);
        for (int a = 0; a < nx; a++)
            for (int b = 0; b < ny; b++) lookups_ += P.query(rx[a][0], rx[a][1], ry[b][0], ry[b][1], blo, bhi);
        return true;
    }
    // band height: ~16 bands over the triangle, a power of two
    int s = 1;
    while (s < 64 && (double)(2 * s) * 16.0 <= yhi - ylo) s *= 2;
    // the triangle's x-extent over y in [a, b]
    auto extent = [&](double a, double b, double& e0, double& e1) {
        e0 = INFINITY, e1 = -INFINITY;
        for (int k = 0; k < 3; k++) {
            if (py[k] >= a && py[k] <= b) e0 = std::min(e0, px[k]), e1 = std::max(e1, px[k]);
            const int m = (k + 1) % 3;
            for (double yy : {a, b}) {
                const double d = py[m] - py[k];
                if (d == 0.0) continue;
                const double t = (yy - py[k]) / d;
                if (t < 0.0 || t > 1.0) continue;
                const double xx = px[k] + t * (px[m] - px[k]);
                e0 = std::min(e0, xx), e1 = std::max(e1, xx);
            }
        }
        return e0 <= e1;
    };
    // rows r0 .. r0 + s - 1 are floor(y) for y in [r0, r0 + s); their
    // bilinear lookups read rows r0 .. r0 + s
    for (int64_t r0 = (int64_t)std::floor(ylo); (double)r0 <= yhi; r0 += s) {
        double e0, e1;
        if (!extent(std::max((double)r0, ylo) - my, std::min((double)(r0 + s), yhi) + my, e0, e1)) continue;
        const int64_t X0 = (int64_t)std::floor(e0 - mx), X1 = (int64_t)std::floor(e1 + mx) + 1;
        int rx[2][2], ry[2][2];
        const int nx = wrap_ranges(X0, X1, P.W, rx), ny = wrap_ranges(r0, r0 + s, P.H, ry);
        for (int a = 0; a < nx; a++)
            for (int b = 0; b < ny; b++) lookups_ += P.query(rx[a][0], rx[a][1], ry[b][0], ry[b][1], blo, bhi);
    }
    return true;
}

// the subdivision for a triangle spanning `ext` texels: cells of ~8 texels, 4 .. max_n per side
static int cells_per_side(double ext, int max_n) {
    int n = 4;
    while (n < max_n && ext > 8.0 * n) n *= 2;
    return n;
}

uint32_t PtAlphaCoverage::set(const PtAlphaRecord& rec) {
    PtAlphaRecord r = rec;
    const bool whole = r.mode == M_OPAQUE || r.src == SRC_CONST;  // one verdict for every cell
    if (!whole && r.src != SRC_CH4 && r.src != SRC_CH1) return PT_ALPHA_SET_NONE;
    if (whole) {  // the verdict does not depend on the uvs: one shared set
        for (int k = 0; k < 3; k++) r.su[k] = r.sv[k] = 0.0f;
        r.off = 0, r.W = r.H = r.C = 0;
    }
    std::string key(reinterpret_cast<const char*>(&r), sizeof r);
    if (auto it = memo_.find(key); it != memo_.end()) return it->second;
    uint32_t out = PT_ALPHA_SET_NONE;
    const Pyramid* P = whole ? nullptr : pyramid(r.off, r.W, r.H, r.C, r.src == SRC_CH4 ? 3u : 0u);
    double maxu = 0, maxv = 0, ext = 0;
    bool finite = std::isfinite(r.scale);
    for (int k = 0; k < 3; k++) {
        finite = finite && std::isfinite(r.su[k]) && std::isfinite(r.sv[k]);
        maxu = std::max(maxu, std::fabs((double)r.su[k]));
        maxv = std::max(maxv, std::fabs((double)r.sv[k]));
        const int m = (k + 1) % 3;
        ext = std::max({ext, std::fabs((double)r.su[m] - r.su[k]) * r.W, std::fabs((double)r.sv[m] - r.sv[k]) * r.H});
    }
    const int n = whole ? 4 : cells_per_side(ext, std::min(256, std::max(4, max_n_)));
    const uint32_t wpm = std::max(1, n * n / 32);  // words per mask
    std::vector<uint32_t> acc(wpm, 0), rej(wpm, 0);
    bool any = false;
    if (whole) {
        const double a = r.mode == M_OPAQUE ? 1.0 : (double)r.constant;
        const int k = decide(r.mode, a, a, r.cut);
        if (k) {
            (k == 1 ? acc : rej)[0] = 0xFFFFu;
            any = true;
        }
    } else if (P && finite && lookups_ < PT_ALPHA_LOOKUP_BUDGET && words_.size() + 2 * wpm < (1u << 29)) {
        // texel-space margins: far above the float error of the computed
        // barycentrics' lerp and of u W - 0.5 (a few ulp of max|u| W)
        const double mx = 1e-4 + 1e-5 * (maxu * r.W + 1.0), my = 1e-4 + 1e-5 * (maxv * r.H + 1.0);
        const double h = 1.0 / n;
        for (int j = 0; j < n; j++)
            for (int i = 0; i < n - j; i++)
                for (int up = 0; up < 2; up++) {
                    if (up && i == n - 1 - j) continue;
                    const int cell = j * (2 * n - j) + 2 * i + up;  // pt_device.h alpha_cell
                    // the sub-triangle's corners in units of 1/n barycentric:
                    // lower (i, j) (i+1, j) (i, j+1), upper (i+1, j) (i, j+1) (i+1, j+1)
                    const int cc[3][2] = {{i + up, j}, {i + 1 - up, j + up}, {i + up, j + 1}};
                    double px[3], py[3];
                    for (int k = 0; k < 3; k++) {
                        const double u = cc[k][0] * h, v = cc[k][1] * h, w = 1.0 - u - v;
                        const double tu = u * r.su[0] + v * r.su[1] + w * r.su[2];
                        const double tv = u * r.sv[0] + v * r.sv[1] + w * r.sv[2];
                        px[k] = tu * r.W - 0.5, py[k] = tv * r.H - 0.5;
                    }
                    uint8_t blo = 255, bhi = 0;
                    if (!footprint(*P, px, py, mx, my, blo, bhi)) continue;
                    // u8_unit (pt_shading.h): byte / 255 correctly rounded
                    const double tlo = (double)((float)blo / 255.0f) - 1e-6, thi = (double)((float)bhi / 255.0f) + 1e-6;
                    double lo = tlo, hi = thi;
                    if (r.src == SRC_CH1) {  // colorScale.x * Evaluate(uv).x
                        const double s = r.scale, e = 1e-6 * (std::fabs(s) + 1.0);
                        lo = std::min(s * tlo, s * thi) - e;
                        hi = std::max(s * tlo, s * thi) + e;
                    }
                    const int dcs = decide(r.mode, lo, hi, r.cut);
                    if (dcs) {
                        (dcs == 1 ? acc : rej)[cell >> 5] |= 1u << (cell & 31);
                        any = true;
                    }
                }
    }
    if (any) {
        int ln = 0;
        while ((4 << ln) < n) ln++;
        if (il_ && (words_.size() & 1)) words_.push_back(0);  // 8-B aligned pairs
        out = (uint32_t)words_.size() | (uint32_t)ln << 29;
        if (il_) {
            for (uint32_t k = 0; k < wpm; k++) words_.push_back(acc[k]), words_.push_back(rej[k]);
        } else {
            words_.insert(words_.end(), acc.begin(), acc.end());
            words_.insert(words_.end(), rej.begin(), rej.end());
        }
    }
    memo_.emplace(std::move(key), out);
    return out;
}

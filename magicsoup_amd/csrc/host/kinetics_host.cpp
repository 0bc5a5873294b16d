// Host (OpenMP) kinetics: parameter build from translated tokens and the fused signal integrator.
// CPU counterpart of hip/kinetics.hip; semantics documented in ms_kinetics.h.
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <vector>
#include <stdexcept>

#include "host_common.h"
#include "ms_kinetics.h"

namespace ms_host {

using farr = py::array_t<float, py::array::c_style>;
using iarr = py::array_t<int32_t, py::array::c_style>;

namespace {

// Per-cell parameter view (contiguous rows of the dense (c, P, s) / (c, P) tensors).
struct CellParams {
  const int32_t *N, *Nf, *Nb, *A;
  const float *Kmr, *Kmf, *Kmb, *Vmax, *Ke;
};

// Trajectory of one integration part for one cell (kinetics.py:753-859 with the loop unrolled to
// all kEqIters iterations). Writes the kSnap candidate states to snap[k*s + j] and returns the
// per-iteration "impactful correction" bits.
constexpr int kChunk = 32;  // canonical chunk of the per-signal sums (kinetics.hip kChunk)

unsigned cell_part(const CellParams& q, int np, int s, const float* X0, float trim, int n_iters, float* snap,
                   float* V, float* Va, float* F, unsigned char* fwd, unsigned char* imp, float* cons, float* fs,
                   uint8_t* dec, int dec_stride) {
  // velocities (kinetics.py:771-806). A protein with Vmax' == 0 has V == 0 and contributes nothing
  // to any later stage (no NV, no impact flag), so it is skipped by marking V = 0 early.
  for (int p = 0; p < np; ++p) {
    if (q.Vmax[p] * trim <= 0.0f) {
      V[p] = 0.0f;
      continue;
    }
    const int32_t* nf = q.Nf + (size_t)p * s;
    const int32_t* nb = q.Nb + (size_t)p * s;
    const int32_t* a = q.A + (size_t)p * s;
    const float* kmr = q.Kmr + (size_t)p * s;
    float xf = 1.0f, xb = 1.0f, ar = 1.0f;
    bool anyf = false, anyb = false;
    for (int j = 0; j < s; ++j) {
      if (nf[j] > 0) {
        xf *= ms::ipow(X0[j], nf[j]);
        anyf = true;
      }
      if (nb[j] > 0) {
        xb *= ms::ipow(X0[j], nb[j]);
        anyb = true;
      }
      if (a[j] != 0) {
        float r = ms::ipow(X0[j], a[j]);
        r = r / (r + kmr[j]);
        if (ms::f_isnan(r)) r = 1.0f;
        ar *= r;
      }
    }
    float kf = ms::clean_prod(xf) / q.Kmf[p];
    if (!anyf) kf = 0.0f;
    if (ms::f_isinf(kf)) kf = ms::kMax;
    float kb = ms::clean_prod(xb) / q.Kmb[p];
    if (!anyb) kb = 0.0f;
    if (ms::f_isinf(kb)) kb = ms::kMax;
    if (ms::f_isinf(ar)) ar = ms::kMax;
    const float acat = (kf - kb) / (1.0f + kf + kb);
    float vmax = q.Vmax[p] * trim;
    if (vmax < 0.0f) vmax = 0.0f;
    float v = acat * vmax * ar;
    v = v < ms::kMin ? ms::kMin : (v > ms::kMax ? ms::kMax : v);
    V[p] = v;
  }
  // The per-signal sums over proteins run over the active proteins (Vmax' != 0; an inactive one adds
  // exact zeros) in the device's canonical chunk order (kinetics.hip kChunk): chunks of 32 active
  // proteins, the first from the initial value, the others from 0, added to the total in order.
  thread_local std::vector<int> act;
  act.resize((size_t)np);
  int na = 0;
  for (int p = 0; p < np; ++p)
    if (!(q.Vmax[p] * trim <= 0.0f)) act[na++] = p;
  // negative-concentration guard (kinetics.py:861-879)
  for (int j = 0; j < s; ++j) cons[j] = 0.0f;
  for (int k0 = 0; k0 < na; k0 += kChunk) {
    const int k1 = std::min(k0 + kChunk, na);
    for (int j = 0; j < s; ++j) {
      float part = 0.0f;
      for (int k = k0; k < k1; ++k) {
        const int p = act[k];
        const float nv = (float)q.N[(size_t)p * s + j] * V[p];
        if (nv < 0.0f) part += -nv;
      }
      cons[j] = k0 == 0 ? part : cons[j] + part;
    }
  }
  for (int j = 0; j < s; ++j) {
    float f = X0[j] / cons[j];
    fs[j] = f > 1.0f ? 1.0f : f;
  }
  for (int p = 0; p < np; ++p) {
    const int32_t* n = q.N + (size_t)p * s;
    float fmin = 1.0f;
    bool nan = false;
    for (int j = 0; j < s; ++j) {
      if ((float)n[j] * V[p] < 0.0f) {
        if (ms::f_isnan(fs[j])) nan = true;
        else if (fs[j] < fmin) fmin = fs[j];
      }
    }
    Va[p] = V[p] * (nan ? NAN : fmin);
  }
  // x_j = X0_j + sum_k n_kj * w(k) over the active proteins, canonical chunk order
  auto chunk_sum = [&](float* x, auto&& w_of) {
    for (int j = 0; j < s; ++j) {
      float tot = X0[j];
      for (int k0 = 0; k0 < na; k0 += kChunk) {
        const int k1 = std::min(k0 + kChunk, na);
        float part = k0 == 0 ? tot : 0.0f;
        for (int k = k0; k < k1; ++k) {
          const int p = act[k];
          const int32_t n = q.N[(size_t)p * s + j];
          part = std::fmaf((float)n, w_of(p), part);
        }
        tot = k0 == 0 ? part : tot + part;
      }
      x[j] = tot < 0.0f ? 0.0f : tot;
    }
  };
  // X1 = X0 + sum_p NV_adj (clamped at 0)
  float* x1 = snap;
  chunk_sum(x1, [&](int p) { return Va[p]; });

  // equilibrium damping trajectory (kinetics.py:808-859)
  unsigned bits = 0;
  for (int p = 0; p < np; ++p) {
    F[p] = 1.0f;
    fwd[p] = V[p] > 0.0f;
    imp[p] = std::fabs(V[p]) > 0.1f;
  }
  float inc = 0.5f;
  for (int it = 0; it < n_iters; ++it, inc *= 0.5f) {
    const float* xc = snap + (size_t)it * s;
    float* xn = snap + (size_t)(it + 1) * s;
    for (int p = 0; p < np; ++p) {
      const int32_t* nf = q.Nf + (size_t)p * s;
      const int32_t* nb = q.Nb + (size_t)p * s;
      float pf = 1.0f, pb = 1.0f;
      bool anyf = false, anyb = false;
      for (int j = 0; j < s; ++j) {
        if (nf[j] > 0) {
          pf *= ms::ipow(xc[j], nf[j]);
          anyf = true;
        }
        if (nb[j] > 0) {
          pb *= ms::ipow(xc[j], nb[j]);
          anyb = true;
        }
      }
      pf = anyf ? ms::clean_prod(pf) : 0.0f;
      pb = anyb ? ms::clean_prod(pb) : 0.0f;
      float Q = pb / pf;
      if (ms::f_isnan(Q)) Q = 1.0f;
      else Q = Q < ms::kEps ? ms::kEps : (Q > ms::kMax ? ms::kMax : Q);
      const float qke = Q / q.Ke[p];
      bool low = fwd[p] ? (qke < ms::kLower) : (qke > ms::kUpper);
      if (fwd[p] && F[p] == 1.0f) low = false;
      bool high = fwd[p] ? (qke > ms::kUpper) : (qke < ms::kLower);
      if (!fwd[p] && F[p] == 0.0f) high = false;
      if ((low || high) && imp[p]) bits |= 1u << it;
      if (dec) dec[(size_t)it * dec_stride + p] = (uint8_t)((low ? 1 : 0) | (high ? 2 : 0));
      float f = F[p];
      if (high) f -= inc;
      if (low) f += inc;
      F[p] = f > 1.0f ? 1.0f : (f < 0.0f ? 0.0f : f);
    }
    chunk_sum(xn, [&](int p) { return Va[p] * F[p]; });
  }
  return bits;
}

}  // namespace

// Fused integrate_signals on host. X (c, s) is updated in place. trims: velocity trim factors
// (reference (0.7, 0.2, 0.1)); n_iters: equilibrium iterations (4, or 0 to disable them).
// Returns the list of per-part global iteration masks (for diagnostics / tests). `reduce_mask`
// (optional callable int -> int) turns a part's local mask into the global one (a domain-decomposed
// world ORs the masks of all ranks, reproducing the reference's `torch.any` over the population).
py::list integrate_signals(farr X, iarr N, iarr Nf, iarr Nb, iarr A, farr Kmr, farr Kmf, farr Kmb, farr Vmax,
                           farr Ke, py::object nprot_obj, std::vector<float> trims, int n_iters,
                           py::object reduce_mask, py::object decisions_obj) {
  if (X.ndim() != 2 || N.ndim() != 3) throw std::invalid_argument("X must be (c,s) and N (c,p,s)");
  const int c = (int)X.shape(0), s = (int)X.shape(1), P = (int)N.shape(1);
  if (N.shape(0) < c || N.shape(2) != s) throw std::invalid_argument("param/signal shape mismatch");
  if (n_iters < 0 || n_iters > ms::kEqIters) throw std::invalid_argument("n_iters must be in 0..4");
  const int32_t* nprot = nullptr;
  iarr np_arr;
  if (!nprot_obj.is_none()) {
    np_arr = nprot_obj.cast<iarr>();
    nprot = np_arr.data();
  }
  // decisions (optional, diagnostics / decision-aware oracle tests): uint8 (c, parts, kEqIters, P),
  // bit 0 "low" (factor raised), bit 1 "high" (factor lowered) of every damping iteration
  uint8_t* dec = nullptr;
  py::array_t<uint8_t, py::array::c_style> dec_arr;
  if (!decisions_obj.is_none()) {
    // written in place: an array of another dtype or layout would be converted into a temporary
    // copy and the decisions silently dropped, so only an exact uint8 C-contiguous array is taken
    if (!py::isinstance<py::array_t<uint8_t, py::array::c_style>>(decisions_obj))
      throw std::invalid_argument("decisions must be a C-contiguous uint8 array");
    dec_arr = py::reinterpret_borrow<py::array_t<uint8_t, py::array::c_style>>(decisions_obj);
    if (!dec_arr.writeable()) throw std::invalid_argument("decisions must be writeable");
    if (dec_arr.size() < (py::ssize_t)((size_t)c * trims.size() * ms::kEqIters * P))
      throw std::invalid_argument("decisions buffer too small");
    dec = dec_arr.mutable_data();
  }
  float* x = X.mutable_data();
  std::vector<float> snaps((size_t)c * ms::kSnap * s);
  py::list masks;
  int part = 0;
  for (float trim : trims) {
    unsigned mask = 0;
    {
      py::gil_scoped_release nogil;
#pragma omp parallel reduction(| : mask)
      {
        std::vector<float> V(P), Va(P), F(P), cons(s), fs(s);
        std::vector<unsigned char> fwd(P), imp(P);
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < c; ++i) {
          const size_t o3 = (size_t)i * P * s, o2 = (size_t)i * P;
          CellParams q{N.data() + o3,   Nf.data() + o3,  Nb.data() + o3,   A.data() + o3, Kmr.data() + o3,
                       Kmf.data() + o2, Kmb.data() + o2, Vmax.data() + o2, Ke.data() + o2};
          int np = nprot ? nprot[i] : P;
          if (np > P) np = P;
          uint8_t* d = dec ? dec + (((size_t)i * trims.size() + part) * ms::kEqIters) * P : nullptr;
          mask |= cell_part(q, np, s, x + (size_t)i * s, trim, n_iters, snaps.data() + (size_t)i * ms::kSnap * s,
                            V.data(), Va.data(), F.data(), fwd.data(), imp.data(), cons.data(), fs.data(), d, P);
        }
      }
    }
    if (!reduce_mask.is_none()) mask = reduce_mask(mask).cast<unsigned>();
    {
      py::gil_scoped_release nogil;
      int stop = n_iters;
      for (int it = 0; it < n_iters; ++it)
        if (!(mask & (1u << it))) {
          stop = it;
          break;
        }
#pragma omp parallel for schedule(static)
      for (int i = 0; i < c; ++i)
        std::memcpy(x + (size_t)i * s, snaps.data() + ((size_t)i * ms::kSnap + stop) * s, sizeof(float) * s);
    }
    masks.append(mask);
    ++part;
  }
  return masks;
}

// Parameter build (kinetics.py:561-625) from dense tokens (n, P, D, 5) into rows `rows` of the
// dense parameter tensors (C, Pt, s) / (C, Pt). Proteins P..Pt-1 of each row get the values the
// reference produces for padding (Ke 1, Kmf = Kmb = EPS, Kmr 1, everything else 0).
void build_params(iarr tokens, iarr rows, farr vmax_w, farr km_w, iarr signs, iarr hills, iarr react_M,
                  iarr trnsp_M, iarr eff_M, farr energies, float abs_temp, float gas_const, iarr N, iarr Nf,
                  iarr Nb, iarr A, farr Kmr, farr Kmf, farr Kmb, farr Vmax, farr Ke) {
  const int n = (int)tokens.shape(0), P = (int)tokens.shape(1), D = (int)tokens.shape(2);
  const int Pt = (int)N.shape(1), s = (int)N.shape(2);
  if (P > Pt) throw std::invalid_argument("token proteins exceed parameter capacity");
  const int nw = (int)vmax_w.size(), nk = (int)km_w.size(), nsg = (int)signs.size(), nh = (int)hills.size();
  const int nv = (int)react_M.shape(0);
  if (react_M.shape(1) != s || trnsp_M.shape(1) != s || eff_M.shape(1) != s)
    throw std::invalid_argument("vector maps must have n_signals columns");
  const int32_t* tk = tokens.data();
  const int32_t* rw = rows.data();
  const float *vw = vmax_w.data(), *kw = km_w.data(), *en = energies.data();
  const int32_t *sg = signs.data(), *hl = hills.data(), *RM = react_M.data(), *TM = trnsp_M.data(),
                *EM = eff_M.data();
  int32_t *oN = N.mutable_data(), *oNf = Nf.mutable_data(), *oNb = Nb.mutable_data(), *oA = A.mutable_data();
  float *oKmr = Kmr.mutable_data(), *oKmf = Kmf.mutable_data(), *oKmb = Kmb.mutable_data(),
        *oV = Vmax.mutable_data(), *oKe = Ke.mutable_data();
  auto lut = [](int t, int lim) { return (t >= 0 && t < lim) ? t : 0; };
  py::gil_scoped_release nogil;
#pragma omp parallel
  {
    std::vector<float> kmr_sum(s);
    std::vector<int> kmr_cnt(s);
#pragma omp for schedule(dynamic, 16)
    for (int i = 0; i < n * Pt; ++i) {
      const int ci = i / Pt, p = i % Pt;
      const size_t row = (size_t)rw[ci];
      int32_t* n_ = oN + (row * Pt + p) * s;
      int32_t* nf_ = oNf + (row * Pt + p) * s;
      int32_t* nb_ = oNb + (row * Pt + p) * s;
      int32_t* a_ = oA + (row * Pt + p) * s;
      float* kmr_ = oKmr + (row * Pt + p) * s;
      for (int j = 0; j < s; ++j) {
        n_[j] = nf_[j] = nb_[j] = a_[j] = 0;
        kmr_sum[j] = 0.0f;
        kmr_cnt[j] = 0;
      }
      ms::NanMean vm, km;
      if (p < P) {
        const int32_t* pt = tk + ((size_t)ci * P + p) * D * 5;
        for (int d = 0; d < D; ++d) {
          const int32_t* dm = pt + d * 5;
          const int t = dm[0];
          if (t == 0) continue;
          const bool reg = t == 3;
          const int sgn = sg[lut(dm[3], nsg)];
          const float kmv = kw[lut(dm[2], nk)];
          if (reg) {
            const int h = hl[lut(dm[1], nh)];
            const int32_t* e = EM + (size_t)lut(dm[4], nv) * s;
            for (int j = 0; j < s; ++j) {
              if (e[j] == 0) continue;
              a_[j] += e[j] * sgn * h;
              const float kv = (float)e[j] * kmv;
              if (!ms::f_isnan(kv) && kv != 0.0f) {
                kmr_sum[j] += kv;
                kmr_cnt[j] += 1;
              }
            }
          } else {
            vm.add(vw[lut(dm[1], nw)]);
            km.add(kmv);
            const int32_t* v = (t == 1 ? RM : TM) + (size_t)lut(dm[4], nv) * s;
            for (int j = 0; j < s; ++j) {
              const int nd = v[j] * sgn;
              n_[j] += nd;
              if (nd < 0) nf_[j] += -nd;
              if (nd > 0) nb_[j] += nd;
            }
          }
        }
      }
      // integer N times float energies, summed in double: exact, so independent of the order
      // (the device reduces it across lanes)
      double E = 0.0;
      for (int j = 0; j < s; ++j) {
        const float km_mean = kmr_cnt[j] > 0 ? kmr_sum[j] / (float)kmr_cnt[j] : 0.0f;
        kmr_[j] = ms::ipow(km_mean, a_[j]);  // (the device build computes the same products)
        E += (double)n_[j] * (double)en[j];
      }
      float ke = (float)std::exp((double)(-(float)E / abs_temp / gas_const));  // (as the device build)
      ke = ke < ms::kEps ? ms::kEps : (ke > ms::kMax ? ms::kMax : ke);
      const float kmn = km.value0();
      float kmf = ke >= 1.0f ? kmn : kmn / ke;
      float kmb = ke >= 1.0f ? kmn * ke : kmn;
      kmf = kmf < ms::kEps ? ms::kEps : (kmf > ms::kMax ? ms::kMax : kmf);
      kmb = kmb < ms::kEps ? ms::kEps : (kmb > ms::kMax ? ms::kMax : kmb);
      const size_t o2 = row * Pt + p;
      oKe[o2] = ke;
      oKmf[o2] = kmf;
      oKmb[o2] = kmb;
      oV[o2] = vm.value0();
    }
  }
}

void bind_kinetics(py::module_& m) {
  m.def("integrate_signals", &integrate_signals, py::arg("X"), py::arg("N"), py::arg("Nf"), py::arg("Nb"),
        py::arg("A"), py::arg("Kmr"), py::arg("Kmf"), py::arg("Kmb"), py::arg("Vmax"), py::arg("Ke"),
        py::arg("nprot"), py::arg("trims"), py::arg("n_iters"), py::arg("reduce_mask") = py::none(),
        py::arg("decisions") = py::none());
  m.def("build_params", &build_params);
}

}  // namespace ms_host

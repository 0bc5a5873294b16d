// gfx950 genome translation over the device genome arena: one wavefront per genome.
//
// The sequential reference scan (rust/genetics.rs:13-123; single-source host version in
// ms_common.h) is reformulated so that all 64 lanes work at once and no lane walks the genome:
//   1. lanes over positions: codon index of every position on both strands -> LDS;
//   2. lanes over positions tabulate the domain type starting at each position; per strand and
//      frame, wave suffix-min scans give the next in-frame stop and the next in-frame domain start
//      of every position;
//   3. lanes over start codons: the CDS end is one lookup; CDSs long enough go into a per-strand
//      list (LDS atomic append, order restored next);
//   4. rank every CDS by (stop ascending, start descending) -- exactly the reference's emission
//      order (a stop closes its frame's pending starts latest-first);
//   5. lanes over CDSs in that order: domain extraction, jumping from domain to domain through the
//      next-domain table (count pass: #domains + "has a catalytic or transporter domain"; write
//      pass: tokens at the protein's slot, from a wave prefix sum; the fused pass does both).
// The genome row is staged in LDS with 16-byte loads first, so the per-position work reads LDS only.
// Forward-strand proteins precede reverse-strand ones (rust/genetics.rs:151-175).
#include "hip_common.h"

namespace msd {

constexpr int kGBlock = 256;  // 4 waves -> up to 4 genomes per workgroup
constexpr int kRankMax = 64;  // CDS lists up to this long are ranked by counting, longer ones sorted
constexpr int kSortCap = 8192;  // global-slot pass: CDS lists up to this long are sorted in LDS
constexpr int kLutBytes = 64 * 3 + 16 + 4096 * 2;

struct TransArgs {
  int n, width, gpb, cap, dt_entries;
  int lmax;                    // slot capacity (positions); longer genomes take the global-slot pass
  uint8_t* gslot;              // global slots (long-genome pass) or nullptr (LDS slots)
  const int32_t* list;         // item -> genome index (long-genome pass) or nullptr (identity)
  int32_t *long_list, *long_count;  // LDS count pass: genomes longer than lmax
  bool stage_dt;
  const int64_t* rows;
  const uint8_t* arena;  // genome pool (cell r: lens[r] bytes at arena + off[r])
  const int64_t* off;
  const int32_t* lens;
  const uint8_t *is_start, *is_stop, *one_codon, *dom_type;
  const uint16_t* two_codon;
  int dom_size, dom_type_size;
  int32_t* nprot;   // (2n,) proteins per strand
  int32_t* ndom;    // (2n,) max domains per strand (count pass)
  int32_t* tokens;  // (n, P, D, 5) (write pass)
  int P, D;
  const int* dn;    // optional device item count (<= n; n is then the capacity)
};

// Positions in a slot are 16-bit for genomes below 64 Ki nt and 32-bit above (Wide: the long-genome
// pass of such a width; recombination lets genomes grow past it in long evolving runs):
// cds [2][cap] (q, p) packed in 2 positions | nstop [2][w] pos | order [2][cap] pos | codons [2][w] u8
// | domain type [2][w] u8 | next domain [2][w] pos | counters
constexpr int kWidePositions = 65535;  // a length bound above this takes the 32-bit layout
__host__ __device__ inline size_t slot_bytes_for(int width, int cap, bool wide = false) {
  const size_t ps = wide ? 4 : 2;
  return ((size_t)2 * cap * 2 * ps + (size_t)2 * width * ps + (size_t)2 * cap * ps + (size_t)2 * width * 2 +
          (size_t)2 * width * ps + 16 + 15) &
         ~(size_t)15;
}
template <bool Wide>
struct PosT {
  using pos = uint16_t;
  using pair = uint32_t;
  static constexpr int kShift = 16;
  static constexpr int kNone = 0xFFFF;  // no stop / no domain (positions stay below it)
};
template <>
struct PosT<true> {
  using pos = uint32_t;
  using pair = uint64_t;
  static constexpr int kShift = 32;
  static constexpr int kNone = 0x7FFFFFFF;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// kT: threads per genome -- one wave (LDS pass: up to four genomes per workgroup) or a whole
// workgroup of kLongT (global-slot pass: one long genome per workgroup; one wave per genome left a
// long evolving run's few genomes of 10^4..10^5 nt latency-bound on serial global-memory loops)
template <bool kCount, bool kWrite, bool Wide = false, int kT = 64>
__global__ void __launch_bounds__(kT > 64 ? kT : kGBlock) translate_kernel(TransArgs a) {
  constexpr bool kBlk = kT > 64;
  constexpr int kNw = kT / 64;  // waves per genome
  using pos_t = typename PosT<Wide>::pos;
  using pair_t = typename PosT<Wide>::pair;
  constexpr int kNone = PosT<Wide>::kNone;
  constexpr int kSh = PosT<Wide>::kShift;
  constexpr pair_t kLo = ((pair_t)1 << kSh) - 1;
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wid = kBlk ? 0 : wv;                  // genome of the workgroup
  const int t = kBlk ? (int)threadIdx.x : lane;  // thread within the genome's group
  auto gsync = [] {
    if constexpr (kBlk) __syncthreads();
    else wave_sync();
  };
  __shared__ int s_aux[kBlk ? 2 + 2 * 6 * kNw + 3 * kNw : 1];  // counters | chunk minima | counts, maxima
  uint8_t* l_start = sm;
  uint8_t* l_stop = sm + 64;
  uint8_t* l_one = sm + 128;
  const uint16_t* l_two = reinterpret_cast<const uint16_t*>(sm + 64 * 3 + 16);
  uint8_t* l_dt = sm + kLutBytes;
  const int dt_bytes = a.stage_dt ? ((a.dt_entries + 15) & ~15) : 0;
  // per-wave slot: CDS lists [2][cap] u32, next stop [2][lmax] u16, emission order [2][cap] u16,
  // codons [2][lmax] u8, domain type at position [2][lmax] u8, counters
  const size_t slot_bytes = slot_bytes_for(a.lmax, a.cap, Wide);
  const int item = blockIdx.x * a.gpb + wid;
  const int n_eff = a.dn ? min(*a.dn, a.n) : a.n;
  if ((int)blockIdx.x * a.gpb >= n_eff) return;  // whole block past the device count
  uint8_t* slot = a.gslot ? a.gslot + (size_t)item * slot_bytes
                          : sm + kLutBytes + dt_bytes + (size_t)wid * slot_bytes;
  const int LW = a.lmax;
  pair_t* cds = reinterpret_cast<pair_t*>(slot);  // (q << kSh) | p
  pos_t* nstop = reinterpret_cast<pos_t*>(cds + 2 * a.cap);
  pos_t* order = nstop + 2 * LW;
  uint8_t* cod = reinterpret_cast<uint8_t*>(order + 2 * a.cap);
  uint8_t* dtp = cod + 2 * LW;
  pos_t* nxd = reinterpret_cast<pos_t*>(dtp + 2 * LW);
  int* counters = kBlk ? s_aux : reinterpret_cast<int*>(nxd + 2 * LW);

  for (int i = threadIdx.x; i < 64; i += blockDim.x) {
    l_start[i] = a.is_start[i];
    l_stop[i] = a.is_stop[i];
    l_one[i] = a.one_codon[i];
  }
  for (int i = threadIdx.x; i < 4096 * 2 / 16; i += blockDim.x)
    reinterpret_cast<uint4*>(sm + 64 * 3 + 16)[i] = reinterpret_cast<const uint4*>(a.two_codon)[i];
  if (a.stage_dt)
    for (int i = threadIdx.x; i < dt_bytes / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(l_dt)[i] = reinterpret_cast<const uint4*>(a.dom_type)[i];
  const uint8_t* DT = a.stage_dt ? l_dt : a.dom_type;

  const bool active = wid < a.gpb && item < n_eff;
  const int g = active ? (a.list ? a.list[item] : item) : 0;
  int L = 0;
  const uint8_t* s = nullptr;
  if (active) {
    const int64_t r = a.rows[g];
    L = a.lens[r];
    s = a.arena + a.off[r];
    if (t < 2) counters[t] = 0;
  }
  __syncthreads();
  if (!active) return;  // whole waves only (one genome per workgroup with kBlk: uniform there)
  if (L > LW) {         // LDS pass: too long for a slot -> queued for the global-slot pass
    if (kCount && t == 0) a.long_list[atomicAdd(a.long_count, 1)] = g;
    return;
  }
  gsync();

  // ---- 0. stage the genome in LDS (16-byte loads: pool allocations are 16-byte aligned and
  //         rounded up; the staging area -- the domain-type table, filled in step 2 -- holds
  //         2 * LW >= L rounded up)
  uint8_t* raw = dtp;
  for (int i = t * 16; i < L; i += kT * 16)
    *reinterpret_cast<uint4*>(raw + i) = *reinterpret_cast<const uint4*>(s + i);
  gsync();

  // ---- 1. codon index per position, both strands (0xFF past the end)
  const int ncod = L - 2;
  for (int i = t; i < L; i += kT) {
    uint8_t cf = 0xFF, cr = 0xFF;
    if (i < ncod) {
      cf = (uint8_t)((ms::nt_code(raw[i]) << 4) | (ms::nt_code(raw[i + 1]) << 2) | ms::nt_code(raw[i + 2]));
      // reverse-complement position i covers forward bases L-1-i, L-2-i, L-3-i
      cr = (uint8_t)((ms::nt_comp(ms::nt_code(raw[L - 1 - i])) << 4) |
                     (ms::nt_comp(ms::nt_code(raw[L - 2 - i])) << 2) | ms::nt_comp(ms::nt_code(raw[L - 3 - i])));
    }
    cod[i] = cf;
    cod[LW + i] = cr;
  }
  gsync();

  // ---- 2. domain type starting at every position; then, per strand and frame, the next in-frame
  //         stop and the next in-frame domain start at or after every position (suffix-min scans;
  //         0xFFFF = none)
  const int ds = a.dom_size, dts = a.dom_type_size, ntc = dts / 3;
  for (int st = 0; st < 2; ++st) {
    const uint8_t* c = cod + st * LW;
    uint8_t* dt = dtp + st * LW;
    for (int p = t; p < L; p += kT) {
      uint8_t ty = 0;
      if (p + dts <= L) {
        int idx = 0;
        for (int t = 0; t < ntc; ++t) idx = (idx << 6) | c[p + 3 * t];
        ty = DT[idx];
      }
      dt[p] = ty;
    }
  }
  gsync();
  // (a workgroup per genome: each wave scans its own contiguous chunk of every strand / frame
  // sequence, then takes the minima of the chunks after it in a second pass)
  int* cmin = s_aux + 2;
  for (int sf = 0; sf < 6; ++sf) {
    const int st = sf / 3, f = sf - 3 * st;
    const uint8_t* c = cod + st * LW;
    const uint8_t* dt = dtp + st * LW;
    pos_t* ns = nstop + st * LW;
    pos_t* nd = nxd + st * LW;
    const int nf = ncod > f ? (ncod - f + 2) / 3 : 0;  // positions f, f+3, ... < ncod
    const int cs = kBlk ? (nf + kNw - 1) / kNw : nf;
    const int lo = kBlk ? min(wv * cs, nf) : 0, top = kBlk ? min(lo + cs, nf) : nf;
    int carry = kNone, carry_d = kNone;
    for (int hi = top; hi > lo; hi -= 64) {
      const int e = hi - 64 + lane;
      const int pe = f + 3 * e;
      int v = (e >= lo && l_stop[c[pe]]) ? pe : kNone;
      int w = (e >= lo && dt[pe]) ? pe : kNone;
      for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_down(v, off), x = __shfl_down(w, off);
        if (lane + off < 64) {
          v = min(v, u);
          w = min(w, x);
        }
      }
      v = min(v, carry);
      w = min(w, carry_d);
      if (e >= lo) {
        ns[pe] = (pos_t)v;
        nd[pe] = (pos_t)w;
      }
      carry = __shfl(v, 0);
      carry_d = __shfl(w, 0);
    }
    if constexpr (kBlk) {
      if (lane == 0) {
        cmin[(2 * sf) * kNw + wv] = carry;
        cmin[(2 * sf + 1) * kNw + wv] = carry_d;
      }
    }
  }
  if constexpr (kBlk) {
    __syncthreads();
    for (int sf = 0; sf < 6; ++sf) {
      const int st = sf / 3, f = sf - 3 * st;
      pos_t* ns = nstop + st * LW;
      pos_t* nd = nxd + st * LW;
      const int nf = ncod > f ? (ncod - f + 2) / 3 : 0;
      const int cs = (nf + kNw - 1) / kNw;
      const int lo = min(wv * cs, nf), top = min(lo + cs, nf);
      int cv = kNone, cd = kNone;
      for (int w = wv + 1; w < kNw; ++w) {
        cv = min(cv, cmin[(2 * sf) * kNw + w]);
        cd = min(cd, cmin[(2 * sf + 1) * kNw + w]);
      }
      if (cv == kNone && cd == kNone) continue;
      for (int e = lo + lane; e < top; e += 64) {
        const int pe = f + 3 * e;
        ns[pe] = (pos_t)min((int)ns[pe], cv);
        nd[pe] = (pos_t)min((int)nd[pe], cd);
      }
    }
  }
  gsync();

  // ---- 3. CDS candidates: start codon -> first in-frame stop (too short / unstopped: dropped)
  if (L >= a.dom_size && L >= 3) {
    for (int st = 0; st < 2; ++st) {
      const uint8_t* c = cod + st * LW;
      const pos_t* ns = nstop + st * LW;
      for (int p = t; p < ncod; p += kT) {
        if (!l_start[c[p]]) continue;
        const int q = p + 3 < ncod ? (int)ns[p + 3] : kNone;
        if (q == kNone || q + 3 - p < a.dom_size) continue;
        const int k = atomicAdd(&counters[st], 1);
        cds[st * a.cap + k] = ((pair_t)q << kSh) | (pair_t)p;  // k < ncod <= cap
      }
    }
  }
  gsync();

  // ---- 4. emission order: stop ascending, start descending, i.e. ascending keys
  //         (stop << kSh) | (kLo - start) -- unique, since every CDS has its own start. Short lists
  //         are ranked by counting (one pass, O(n^2)); long ones (long genomes: hundreds of CDSs,
  //         the quadratic ranking took most of an evolved population's translation time) are sorted
  //         in place by an all-ascending bitonic network (mirrored first comparison per stage, so
  //         positions past n act as +inf and need no padding), and phase 5 decodes the keys.
  int ncds[2];
  bool keyed[2];
  for (int st = 0; st < 2; ++st) {
    ncds[st] = counters[st];
    const int n = ncds[st];
    pair_t* lst = cds + st * a.cap;
    keyed[st] = n > kRankMax;
    if (!keyed[st]) {
      for (int e = t; e < n; e += kT) {
        const pair_t ve = lst[e];
        const pair_t ke = (ve & ~kLo) | (kLo - (ve & kLo));
        int rank = 0;
        for (int f = 0; f < n; ++f) {
          const pair_t vf = lst[f];
          rank += ((vf & ~kLo) | (kLo - (vf & kLo))) < ke;
        }
        order[st * a.cap + rank] = (pos_t)e;
      }
      continue;
    }
    // (a workgroup per genome sorts lists up to kSortCap in LDS: in its global-memory slot every
    // compare-exchange pass of the network was a load round trip)
    pair_t* const lst_g = lst;
    if constexpr (kBlk) {
      if (n <= kSortCap) lst = reinterpret_cast<pair_t*>(sm + kLutBytes + dt_bytes);
    }
    for (int e = t; e < n; e += kT) {
      const pair_t ve = lst_g[e];
      lst[e] = (ve & ~kLo) | (kLo - (ve & kLo));
    }
    gsync();
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int k = 2; k <= n2; k <<= 1) {
      for (int i = t; i < n2 / 2; i += kT) {  // mirrored pairs of each k-block
        const int blk = i / (k / 2), off = i - blk * (k / 2);
        const int lo = blk * k + off, hi = blk * k + k - 1 - off;
        if (hi < n) {
          const pair_t x = lst[lo], y = lst[hi];
          if (y < x) {
            lst[lo] = y;
            lst[hi] = x;
          }
        }
      }
      gsync();
      for (int j = k / 4; j >= 1; j >>= 1) {  // half-cleaners
        for (int i = t; i < n2 / 2; i += kT) {
          const int blk = i / j, off = i - blk * j;
          const int lo = blk * 2 * j + off, hi = lo + j;
          if (hi < n) {
            const pair_t x = lst[lo], y = lst[hi];
            if (y < x) {
              lst[lo] = y;
              lst[hi] = x;
            }
          }
        }
        gsync();
      }
    }
    if (lst != lst_g) {  // (back to the slot: phase 5 reads it there; the buffer serves the next strand)
      for (int e = t; e < n; e += kT) lst_g[e] = lst[e];
      gsync();
    }
  }
  gsync();

  // ---- 5. domain extraction in emission order
  int prot_base = 0;  // forward-strand proteins come first
  for (int st = 0; st < 2; ++st) {
    const uint8_t* c = cod + st * LW;
    const uint8_t* dt = dtp + st * LW;
    const pos_t* nd_s = nxd + st * LW;
    int n_prot = 0, max_dom = 0;
    for (int e0 = 0; e0 < ncds[st]; e0 += kT) {
      const int e = e0 + t;
      const bool have = e < ncds[st];
      int p = 0, n = 0;
      if (have) {
        if (keyed[st]) {  // (a sorted key: stop, and the start inverted)
          const pair_t k = cds[st * a.cap + e];
          p = (int)(kLo - (k & kLo));
          n = (int)(k >> kSh) + 3 - p;
        } else {
          const pair_t v = cds[st * a.cap + order[st * a.cap + e]];
          p = (int)(v & kLo);
          n = (int)(v >> kSh) + 3 - p;
        }
      }
      // domains of the CDS [p, p + n): from position x, the next one starts at nd_s[x] (same frame;
      // every skipped position has no domain type); it counts if it ends inside the CDS
      const int end = p + n;
      int nd = 0;
      bool useful = false;
      for (int x = p; x < ncod;) {
        x = nd_s[x];
        if (x == kNone || x + ds > end) break;
        useful |= dt[x] != 3;
        ++nd;
        x += ds;
      }
      const unsigned long long bal = __ballot(useful);
      int rank = __popcll(bal & ((1ull << lane) - 1ull)), emitted = __popcll(bal);
      if constexpr (kBlk) {  // (the waves' proteins in wave order)
        int* wcnt = s_aux + 2 + 12 * kNw;
        if (lane == 0) wcnt[wv] = emitted;
        __syncthreads();
        emitted = 0;
        for (int w = 0; w < kNw; ++w) {
          const int x = wcnt[w];
          rank += w < wv ? x : 0;
          emitted += x;
        }
        __syncthreads();
      }
      if constexpr (kWrite) {
        const int slot_p = prot_base + n_prot + rank;
        if (useful && slot_p < a.P) {
          int32_t* tk = a.tokens + ((size_t)g * a.P + slot_p) * a.D * 5;
          int d = 0;
          for (int x = p; x < ncod && d < a.D;) {
            x = nd_s[x];
            if (x == kNone || x + ds > end) break;
            const int o = x + dts;
            int32_t* dm = tk + d * 5;
            dm[0] = dt[x];
            dm[1] = l_one[c[o]];
            dm[2] = l_one[c[o + 3]];
            dm[3] = l_one[c[o + 6]];
            dm[4] = l_two[((int)c[o + 9] << 6) | c[o + 12]];
            ++d;
            x += ds;
          }
        }
      }
      if constexpr (kCount) {
        if (useful && nd > max_dom) max_dom = nd;
      }
      n_prot += emitted;
    }
    if constexpr (kCount) {
      for (int o = 32; o > 0; o >>= 1) max_dom = max(max_dom, __shfl_xor(max_dom, o));
      if constexpr (kBlk) {
        int* wmax = s_aux + 2 + 12 * kNw + (1 + st) * kNw;
        if (lane == 0) wmax[wv] = max_dom;
        __syncthreads();
        for (int w = 0; w < kNw; ++w) max_dom = max(max_dom, wmax[w]);
      }
      if (t == 0) {
        a.nprot[2 * g + st] = n_prot;
        a.ndom[2 * g + st] = max_dom;
      }
    }
    prot_base += n_prot;
  }
}

// genomes up to this length use LDS slots (24 B per nt and strand pair: 2048 nt = 49 KB, one wave per
// workgroup, three workgroups per CU); longer ones go to the global-slot pass. At 1024 the genomes
// of a long flagship run (lengths grow past 1024 after a few hundred steps) took the global pass,
// 100 us per chain under the diffusion stencil (profiles/r4/s17/tlong_steps.txt)
constexpr int kLdsMaxLen = 2048;
int translate_lds_max() { return kLdsMaxLen; }
constexpr int kLongT = 1024;  // threads per genome of the global-slot pass

// mode: 0 count pass, 1 write pass, 2 fused (counts and tokens; the caller checks the counts
// against P / D afterwards)
static void launch(int mode, int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens,
                   uintptr_t luts,
                   uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                   uintptr_t nprot, uintptr_t ndom, int P, int D, uintptr_t tokens, uintptr_t list, uintptr_t gslot,
                   uintptr_t long_list, uintptr_t long_count, uintptr_t dn, uintptr_t stream) {
  if (n <= 0) return;
  if (width % 16 != 0) throw std::invalid_argument("genome length bound must be a multiple of 16");
  if (!off) throw std::invalid_argument("translate: genome offsets required");
  if (width > (1 << 30)) throw std::invalid_argument("genomes longer than 2^30 nt are not supported on the GPU");
  TransArgs a{};
  a.n = n;
  a.width = width;
  a.dt_entries = dt_entries;
  a.rows = P_<int64_t>(rows);
  a.arena = P_<uint8_t>(arena);
  a.off = P_<int64_t>(off);
  a.lens = P_<int32_t>(lens);
  const uint8_t* l = P_<uint8_t>(luts);  // is_start | is_stop | one_codon (64 bytes each)
  a.is_start = l;
  a.is_stop = l + 64;
  a.one_codon = l + 128;
  a.dom_type = P_<uint8_t>(dom_type);
  a.two_codon = P_<uint16_t>(two_codon);
  a.dom_size = dom_size;
  a.dom_type_size = dom_type_size;
  a.nprot = P_<int32_t>(nprot);
  a.ndom = P_<int32_t>(ndom);
  a.tokens = P_<int32_t>(tokens);
  a.P = P;
  a.D = D;
  a.stage_dt = dt_entries <= 4096;
  a.list = list ? P_<int32_t>(list) : nullptr;
  a.gslot = gslot ? P_<uint8_t>(gslot) : nullptr;
  a.long_list = P_<int32_t>(long_list);
  a.long_count = P_<int32_t>(long_count);
  a.dn = dn ? P_<int>(dn) : nullptr;
  // LDS pass: slots for genomes up to kLdsMaxLen (longer ones are queued); global pass: whole width
  a.lmax = a.gslot ? width : (width < kLdsMaxLen ? width : kLdsMaxLen);
  a.cap = a.lmax;  // a strand has at most one CDS per codon position
  const bool wide = a.lmax > kWidePositions;  // (only the global-slot pass of a length bound past 64 Ki)
  const size_t fixed = kLutBytes + (a.stage_dt ? ((dt_entries + 15) & ~15) : 0);
  const size_t slot = slot_bytes_for(a.lmax, a.cap, wide);
  int gpb = kGBlock / 64;
  if (!a.gslot) {
    while (gpb > 1 && fixed + gpb * slot > 64 * 1024) --gpb;
    if (fixed + gpb * slot > 160 * 1024) throw std::invalid_argument("translation slot does not fit in LDS");
  } else {
    gpb = 1;  // one genome per workgroup of kLongT threads
  }
  a.gpb = gpb;
  const size_t lds = fixed + (a.gslot ? (size_t)kSortCap * (wide ? 8 : 4) : gpb * slot);
  const unsigned grid = cdiv(n, gpb);
  hipStream_t st = S_(stream);
  if (a.gslot) {
    constexpr int T = kLongT;
    if (wide) {
      if (mode == 0) msd::kl(translate_kernel<true, false, true, T>, grid, T, lds, st)(a);
      else if (mode == 1) msd::kl(translate_kernel<false, true, true, T>, grid, T, lds, st)(a);
      else msd::kl(translate_kernel<true, true, true, T>, grid, T, lds, st)(a);
    } else if (mode == 0) {
      msd::kl(translate_kernel<true, false, false, T>, grid, T, lds, st)(a);
    } else if (mode == 1) {
      msd::kl(translate_kernel<false, true, false, T>, grid, T, lds, st)(a);
    } else {
      msd::kl(translate_kernel<true, true, false, T>, grid, T, lds, st)(a);
    }
  } else if (mode == 0) {
    msd::kl(translate_kernel<true, false>, grid, gpb * 64, lds, st)(a);
  } else if (mode == 1) {
    msd::kl(translate_kernel<false, true>, grid, gpb * 64, lds, st)(a);
  } else {
    msd::kl(translate_kernel<true, true>, grid, gpb * 64, lds, st)(a);
  }
  MS_LAUNCH_CHECK();
}

size_t translate_slot_bytes(int width) { return slot_bytes_for(width, width, width > kWidePositions); }

// n items; list: item -> genome index into rows (0 = identity); gslot: global slots for the
// long-genome pass (n * translate_slot_bytes(width) bytes) or 0 for the LDS pass, which queues
// genomes longer than its slots in long_list / long_count.
void translate_count(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, uintptr_t ndom, uintptr_t list, uintptr_t gslot, uintptr_t long_list,
                     uintptr_t long_count, uintptr_t dn, uintptr_t stream) {
  launch(0, n, rows, arena, off, width, lens, luts, dom_type, dt_entries, two_codon, dom_size, dom_type_size, nprot,
         ndom, 0, 0, 0, list, gslot, long_list, long_count, dn, stream);
}

void translate_write(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, int P, int D, uintptr_t tokens, uintptr_t list, uintptr_t gslot,
                     uintptr_t dn, uintptr_t stream) {
  launch(1, n, rows, arena, off, width, lens, luts, dom_type, dt_entries, two_codon, dom_size, dom_type_size, nprot, 0,
         P, D, tokens, list, gslot, 0, 0, dn, stream);
}

// Count and write in one launch (LDS pass): tokens for up to P proteins / D domains each, plus the
// per-strand counts and the long-genome queue of the count pass.
void translate_fused(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, uintptr_t ndom, int P, int D, uintptr_t tokens, uintptr_t long_list,
                     uintptr_t long_count, uintptr_t dn, uintptr_t stream) {
  launch(2, n, rows, arena, off, width, lens, luts, dom_type, dt_entries, two_codon, dom_size, dom_type_size, nprot, ndom,
         P, D, tokens, 0, 0, long_list, long_count, dn, stream);
}

// Long-genome pass of the fused translation with a device count: the items long_list[0..*dn)
// (at most lcap) take global-memory slots (lcap * translate_slot_bytes(width) bytes at gslot).
void translate_fused_long(int lcap, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                          uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                          uintptr_t nprot, uintptr_t ndom, int P, int D, uintptr_t tokens, uintptr_t long_list,
                          uintptr_t gslot, uintptr_t dn, uintptr_t stream) {
  launch(2, lcap, rows, arena, off, width, lens, luts, dom_type, dt_entries, two_codon, dom_size, dom_type_size, nprot, ndom,
         P, D, tokens, long_list, gslot, 0, 0, dn, stream);
}

}  // namespace msd

// sp_roles.hip -- the roles PackedOutputStream.write gives the words of one
// 64-word step, as scalar mask algebra over the step's Z / D-or-L / D masks
// and the run state entering it (SpSt, sp_roles), and the lane helpers the
// single pass uses with them (readfirstlane / readlane / writelane pairs,
// v_ffbl, per-lane selects on an SGPR mask).  Included by encode_v4.hip
// (in namespace cpk, for the single pass) and, for the single pass's sparse
// form (a second namespace), again by encode_sp.hip.

struct SpSt {
  uint32_t zl;   // zero run ending at the step start (0: none)
  uint32_t dlo;  // the word before the step is a D/L word
  uint32_t hd;   // distance back to that stretch's last 0xFF head (0: none), <= 256
};

__device__ __forceinline__ uint64_t sp_uni(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t sp_rl(uint32_t lo, uint32_t hi, int j) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, j) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, j) << 32);
}
// v_writelane_b32 (the LLVM intrinsic; clang exposes no builtin for it)
extern "C" __device__ int cpk_llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t sp_wl(uint32_t old, uint32_t v, int j) {
  return (uint32_t)cpk_llvm_writelane((int)v, j, (int)old);
}
// index of the lowest set bit, 0xffffffff for 0 (v_ffbl_b32)
__device__ __forceinline__ uint32_t sp_ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// per lane: mask bit set ? b : a (one v_cndmask on the SGPR mask)
__device__ __forceinline__ uint32_t sp_sel(uint32_t a, uint32_t b, uint64_t mask) {
  uint32_t r;
  asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mask));
  return r;
}

// Roles of one step from its masks and the state entering it; the state
// entering the next step replaces st (tools/step_model.py: roles).
__device__ __forceinline__ void sp_roles(uint64_t Z, uint64_t DL, uint64_t D, SpSt &st,
                                         uint64_t &Zh, uint64_t &Mem) {
  // zero runs: a head at each run start and every 256 words after it
  Zh = Z & ~((Z << 1) | (st.zl ? 1ull : 0ull));
  if (st.zl && (Z & 1)) {
    const uint32_t j0 = (256u - (st.zl & 255u)) & 255u;
    if (j0 < 64) {
      const uint64_t pre = j0 == 63 ? ~0ull : ((2ull << j0) - 1);
      if ((Z & pre) == pre) Zh |= 1ull << j0;
    }
  }
  const uint64_t nz = ~Z;
  const uint32_t zl2 = nz ? (uint32_t)__builtin_clzll(nz) : st.zl + 64;
  // D/L stretches: each head's literal run covers up to 255 following words
  if (st.dlo && (DL & 1) && st.hd >= 193) {
    // the carried head's coverage ends inside this step: the next head is
    // the first D >= that head + 256 (:143-161)
    const uint64_t ndl = ~DL;
    const int f = ndl ? __builtin_ctzll(ndl) : 64;
    const uint64_t rng = f >= 64 ? ~0ull : ((1ull << f) - 1);
    const uint64_t A = (D << 1) & DL;
    const uint64_t C = (DL + A) ^ DL ^ A;
    Mem = DL & (A | C) & ~rng;
    const int c = 255 - (int)st.hd;
    uint64_t cm = 0;
    if (c >= 0) {
      const int k = min(c + 1, f);
      cm = k >= 64 ? ~0ull : ((1ull << k) - 1);
    }
    const int x = max(c + 1, 0);
    const uint64_t dc = x >= 64 ? 0ull : (D & rng & (~0ull << x));
    if (dc) {
      const int h1 = __builtin_ctzll(dc);
      cm |= rng & (h1 >= 63 ? 0ull : (~0ull << (h1 + 1)));
    }
    Mem |= cm;
  } else {
    const uint64_t cin = (st.dlo && (DL & 1) && st.hd) ? 1ull : 0ull;
    const uint64_t A = ((D << 1) | cin) & DL;
    const uint64_t C = (DL + A) ^ DL ^ A;
    Mem = DL & (A | C);
  }
  uint32_t hd2 = 0, dlo2 = 0;
  if (DL >> 63) {
    dlo2 = 1;
    const uint64_t nd = ~DL;
    const int t = nd ? 64 - __builtin_clzll(nd) : 0;  // start of the run reaching bit 63
    const uint64_t H = D & ~Mem & (~0ull << t);
    if (H) hd2 = 1u + (uint32_t)__builtin_clzll(H);
    else if (t == 0 && st.dlo && st.hd) hd2 = min(st.hd + 64u, 256u);
  }
  st.zl = zl2;
  st.dlo = dlo2;
  st.hd = hd2;
}


// Does an LDS-DMA read its address VGPRs at issue?  (VERDICT r04 "Weak" 1)
//
// tools/dma_hazard_scan.py lists product-kernel sites where hipcc gives a
// ds_read the destination registers of a global_load_lds that is still in
// flight (no vmcnt wait between them).  If the DMA read its address after the
// LDS return landed, it would fetch from whatever the ds_read returned.  This
// probe makes that happen on purpose and counts the outcome, per DMA form:
//
//   form 0  global_load_lds_dwordx4 v[a:a+1], off   (64-bit vaddr: the only
//           form in libmde_hip) followed IMMEDIATELY by ds_read_b64 v[a:a+1]
//           returning a valid DECOY address (another part of the same buffer)
//   form 1  global_load_lds_dwordx4 v_off, s[base]  (SADDR, 32-bit offset)
//           followed immediately by ds_read_b32 v_off returning a decoy offset
//   form 2  buffer_load_dwordx4 v_off, s[rsrc], 0 offen lds, then
//           ds_read_b32 v_off (decoy offset)
//   form 3  form 0 with a VALU overwrite (v_mov_b64) instead of the ds_read --
//           what every compiled kernel does right after a VMEM issue
//   form 4  POSITIVE CONTROL: the decoy is loaded into the address registers
//           BEFORE the DMA, so every lane must see decoy data (proves the
//           checker detects a late address read)
//
// Four DMAs are issued back to back per iteration (each followed by its own
// overwrite), from 8 workgroups x 4 waves per CU, over a 1 GiB source so most
// fetches miss L2/MALL and the TA queues stay full.  Each lane then reads its
// 16 B of every slot and compares with the unique word pattern of the address
// it asked for (word i of the buffer holds i).  Both addresses are always
// valid: a late read gives wrong data, never a fault.  Everything touching the
// registers is one asm block, so the compiler cannot move or re-allocate
// anything in between.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/dma_war_probe tools/dma_war_probe.hip
//   ./build/dma_war_probe [iters] [launches]   -> one JSON line
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int NW = 4;                 // waves per workgroup
constexpr int ND = 4;                 // DMAs in flight per wave per iteration
constexpr size_t SRC_BYTES = 1ull << 30;
constexpr size_t UNITS = SRC_BYTES / 1024;  // 1 KiB = one wave-instruction

__global__ void fill(u32x4* s, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned w = (unsigned)(4 * i);
    s[i] = u32x4{w, w + 1, w + 2, w + 3};
  }
}

template <int FORM>
__global__ __launch_bounds__(NW * 64) void probe(const u32x4* __restrict__ src, int iters, unsigned* __restrict__ bad) {
  __shared__ __attribute__((aligned(1024))) u32x4 slot[NW][ND][64];
  __shared__ __attribute__((aligned(16))) unsigned long long tbl[NW][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const size_t gw = (size_t)blockIdx.x * NW + wave;
  // decoy unit: far from anything this wave asks for
  const size_t decoy_unit = (gw * 7919 + UNITS / 2) % UNITS;
  const unsigned long long decoy_addr = (unsigned long long)(src + decoy_unit * 64 + lane);
  const unsigned decoy_off = (unsigned)(decoy_unit * 1024 + lane * 16);
  if (FORM == 0 || FORM == 3 || FORM == 4) tbl[wave][lane] = decoy_addr;
  else reinterpret_cast<unsigned*>(&tbl[wave][0])[lane] = decoy_off;
  __syncthreads();
  const unsigned tbl_lds = (unsigned)(uintptr_t)(FORM == 0 || FORM == 4 ? (void*)&tbl[wave][lane]
                                                                         : (void*)(reinterpret_cast<unsigned*>(&tbl[wave][0]) + lane));
  const unsigned s0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)&slot[wave][0][0]);
  const unsigned my_slot = (unsigned)(uintptr_t)&slot[wave][0][lane];
  // buffer resource over the whole source (num_records = 1 GiB, raw buffer)
  const unsigned long long base = (unsigned long long)src;
  unsigned nbad = 0;
  size_t u = (gw * 104729) % UNITS;
  for (int it = 0; it < iters; ++it) {
    size_t uu[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) { uu[d] = u; u += 9973; if (u >= UNITS) u -= UNITS; }
    u32x4 r0, r1, r2, r3;
    unsigned keep;
    if constexpr (FORM == 0 || FORM == 3 || FORM == 4) {
      unsigned long long a0 = base + uu[0] * 1024 + lane * 16, a1 = base + uu[1] * 1024 + lane * 16,
                         a2 = base + uu[2] * 1024 + lane * 16, a3 = base + uu[3] * 1024 + lane * 16;
      if constexpr (FORM == 0) {
        asm volatile(
            "s_mov_b32 %[keep], m0\n\t"
            "s_mov_b32 m0, %[s0]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a0], off\n\tds_read_b64 %[a0], %[t]\n\t"
            "s_add_u32 m0, %[s0], 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a1], off\n\tds_read_b64 %[a1], %[t]\n\t"
            "s_add_u32 m0, %[s0], 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a2], off\n\tds_read_b64 %[a2], %[t]\n\t"
            "s_add_u32 m0, %[s0], 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a3], off\n\tds_read_b64 %[a3], %[t]\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
            "ds_read_b128 %[r0], %[ms]\n\tds_read_b128 %[r1], %[ms] offset:1024\n\t"
            "ds_read_b128 %[r2], %[ms] offset:2048\n\tds_read_b128 %[r3], %[ms] offset:3072\n\t"
            "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %[keep]"
            : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3),
              [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [keep] "=&s"(keep)
            : [s0] "s"(s0), [t] "v"(tbl_lds), [ms] "v"(my_slot)
            : "memory");
      } else if constexpr (FORM == 3) {
        asm volatile(
            "s_mov_b32 %[keep], m0\n\t"
            "s_mov_b32 m0, %[s0]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a0], off\n\tv_mov_b64 %[a0], %[dec]\n\t"
            "s_add_u32 m0, %[s0], 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a1], off\n\tv_mov_b64 %[a1], %[dec]\n\t"
            "s_add_u32 m0, %[s0], 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a2], off\n\tv_mov_b64 %[a2], %[dec]\n\t"
            "s_add_u32 m0, %[s0], 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a3], off\n\tv_mov_b64 %[a3], %[dec]\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
            "ds_read_b128 %[r0], %[ms]\n\tds_read_b128 %[r1], %[ms] offset:1024\n\t"
            "ds_read_b128 %[r2], %[ms] offset:2048\n\tds_read_b128 %[r3], %[ms] offset:3072\n\t"
            "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %[keep]"
            : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3),
              [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [keep] "=&s"(keep)
            : [s0] "s"(s0), [dec] "v"(decoy_addr), [ms] "v"(my_slot)
            : "memory");
      } else {  // FORM 4: the decoy lands in the address registers before the DMA
        asm volatile(
            "s_mov_b32 %[keep], m0\n\t"
            "ds_read_b64 %[a0], %[t]\n\tds_read_b64 %[a1], %[t]\n\tds_read_b64 %[a2], %[t]\n\tds_read_b64 %[a3], %[t]\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "s_mov_b32 m0, %[s0]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a0], off\n\t"
            "s_add_u32 m0, %[s0], 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a1], off\n\t"
            "s_add_u32 m0, %[s0], 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a2], off\n\t"
            "s_add_u32 m0, %[s0], 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a3], off\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
            "ds_read_b128 %[r0], %[ms]\n\tds_read_b128 %[r1], %[ms] offset:1024\n\t"
            "ds_read_b128 %[r2], %[ms] offset:2048\n\tds_read_b128 %[r3], %[ms] offset:3072\n\t"
            "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %[keep]"
            : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3),
              [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [keep] "=&s"(keep)
            : [s0] "s"(s0), [t] "v"(tbl_lds), [ms] "v"(my_slot)
            : "memory");
      }
    } else if constexpr (FORM == 1) {
      unsigned o0 = (unsigned)(uu[0] * 1024 + lane * 16), o1 = (unsigned)(uu[1] * 1024 + lane * 16),
               o2 = (unsigned)(uu[2] * 1024 + lane * 16), o3 = (unsigned)(uu[3] * 1024 + lane * 16);
      asm volatile(
            "s_mov_b32 %[keep], m0\n\t"
          "s_mov_b32 m0, %[s0]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[o0], %[b]\n\tds_read_b32 %[o0], %[t]\n\t"
          "s_add_u32 m0, %[s0], 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[o1], %[b]\n\tds_read_b32 %[o1], %[t]\n\t"
          "s_add_u32 m0, %[s0], 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[o2], %[b]\n\tds_read_b32 %[o2], %[t]\n\t"
          "s_add_u32 m0, %[s0], 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[o3], %[b]\n\tds_read_b32 %[o3], %[t]\n\t"
          "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
          "ds_read_b128 %[r0], %[ms]\n\tds_read_b128 %[r1], %[ms] offset:1024\n\t"
          "ds_read_b128 %[r2], %[ms] offset:2048\n\tds_read_b128 %[r3], %[ms] offset:3072\n\t"
          "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %[keep]"
          : [o0] "+v"(o0), [o1] "+v"(o1), [o2] "+v"(o2), [o3] "+v"(o3),
            [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [keep] "=&s"(keep)
          : [s0] "s"(s0), [b] "s"(base), [t] "v"(tbl_lds), [ms] "v"(my_slot)
          : "memory");
    } else {  // FORM 2: MUBUF offen lds
      unsigned o0 = (unsigned)(uu[0] * 1024 + lane * 16), o1 = (unsigned)(uu[1] * 1024 + lane * 16),
               o2 = (unsigned)(uu[2] * 1024 + lane * 16), o3 = (unsigned)(uu[3] * 1024 + lane * 16);
      // raw buffer descriptor: base, stride 0, num_records = 1 GiB, dword3 as
      // the gfx9 raw-buffer default (DATA_FORMAT 32, dst_sel xyzw)
      const u32x4 rsrc = {(unsigned)base, (unsigned)(base >> 32) & 0xffffu, (unsigned)SRC_BYTES, 0x00020000u};
      __attribute__((ext_vector_type(4))) int srs;
      srs[0] = __builtin_amdgcn_readfirstlane((int)rsrc[0]);
      srs[1] = __builtin_amdgcn_readfirstlane((int)rsrc[1]);
      srs[2] = __builtin_amdgcn_readfirstlane((int)rsrc[2]);
      srs[3] = __builtin_amdgcn_readfirstlane((int)rsrc[3]);
      asm volatile(
            "s_mov_b32 %[keep], m0\n\t"
          "s_mov_b32 m0, %[s0]\n\ts_nop 0\n\tbuffer_load_dwordx4 %[o0], %[rs], 0 offen lds\n\tds_read_b32 %[o0], %[t]\n\t"
          "s_add_u32 m0, %[s0], 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %[o1], %[rs], 0 offen lds\n\tds_read_b32 %[o1], %[t]\n\t"
          "s_add_u32 m0, %[s0], 0x800\n\ts_nop 0\n\tbuffer_load_dwordx4 %[o2], %[rs], 0 offen lds\n\tds_read_b32 %[o2], %[t]\n\t"
          "s_add_u32 m0, %[s0], 0xc00\n\ts_nop 0\n\tbuffer_load_dwordx4 %[o3], %[rs], 0 offen lds\n\tds_read_b32 %[o3], %[t]\n\t"
          "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
          "ds_read_b128 %[r0], %[ms]\n\tds_read_b128 %[r1], %[ms] offset:1024\n\t"
          "ds_read_b128 %[r2], %[ms] offset:2048\n\tds_read_b128 %[r3], %[ms] offset:3072\n\t"
          "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %[keep]"
          : [o0] "+v"(o0), [o1] "+v"(o1), [o2] "+v"(o2), [o3] "+v"(o3),
            [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [keep] "=&s"(keep)
          : [s0] "s"(s0), [rs] "s"(srs), [t] "v"(tbl_lds), [ms] "v"(my_slot)
          : "memory");
    }
    const u32x4 rr[ND] = {r0, r1, r2, r3};
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const unsigned w = (unsigned)(4 * (uu[d] * 64 + lane));
      nbad += (rr[d][0] != w) | (rr[d][1] != w + 1) | (rr[d][2] != w + 2) | (rr[d][3] != w + 3);
    }
  }
  bad[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = nbad;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const int launches = argc > 2 ? atoi(argv[2]) : 4;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount * 8;
  u32x4* src;
  unsigned* bad;
  CHECK(hipMalloc(&src, SRC_BYTES));
  CHECK(hipMalloc(&bad, (size_t)grid * NW * 64 * sizeof(unsigned)));
  fill<<<4096, 256>>>(src, SRC_BYTES / 16);
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned> h((size_t)grid * NW * 64);
  const double lane_dmas = (double)grid * NW * 64 * iters * ND * launches;
  printf("{\"probe\": \"lds_dma_address_war\", \"grid\": %d, \"waves_per_wg\": %d, \"dmas_per_iter\": %d, "
         "\"iters\": %d, \"launches\": %d, \"lane_dmas_per_form\": %.0f, \"forms\": {",
         grid, NW, ND, iters, launches, lane_dmas);
  const char* names[5] = {"vaddr64_then_ds_read", "saddr_then_ds_read", "mubuf_lds_then_ds_read",
                          "vaddr64_then_valu", "control_decoy_before_dma"};
  for (int f = 0; f < 5; ++f) {
    unsigned long long total = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int l = 0; l < launches; ++l) {
      switch (f) {
        case 0: probe<0><<<grid, NW * 64>>>(src, iters, bad); break;
        case 1: probe<1><<<grid, NW * 64>>>(src, iters, bad); break;
        case 2: probe<2><<<grid, NW * 64>>>(src, iters, bad); break;
        case 3: probe<3><<<grid, NW * 64>>>(src, iters, bad); break;
        default: probe<4><<<grid, NW * 64>>>(src, iters, bad); break;
      }
      CHECK(hipGetLastError());
      CHECK(hipMemcpy(h.data(), bad, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
      for (unsigned v : h) total += v;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("%s\"%s\": {\"bad_lane_dmas\": %llu, \"seconds\": %.3f, \"GBps\": %.0f}", f ? ", " : "", names[f], total, s,
           lane_dmas * 16 / s / 1e9);
    fflush(stdout);
  }
  printf("}}\n");
  CHECK(hipFree(src));
  CHECK(hipFree(bad));
  return 0;
}

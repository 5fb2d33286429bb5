// smmd_ldsdma.hpp -- the filter-stage LDS-DMA piece shared by the Winograd
// kernels (smmd_wino.hip, smmd_wino_s2.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smmd {

// LDS byte offset of a shared-memory pointer
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)reinterpret_cast<uintptr_t>(
        (const __attribute__((address_space(3))) void *)p);
}

// one 1-KiB LDS-DMA piece: 64 lanes x 16 bytes from sbase + voff into LDS at
// the wave-uniform byte offset lds_dst (lane l at + 16 l).  Written as asm
// because the compiler's own form would make every later LDS read wait for
// it.  Every piece's completion is a vmcnt(0) wait by its issuing wave
// before the stage barrier (dma_wait_all; no partial counts).  The compiler
// does not count these loads, which can only make its own vmcnt(N) waits for
// the row loads wait longer, never shorter.  WN_DMA_SYNC (the `conservative`
// make target, checked bit for bit against the shipped build by
// tools/lib_bitexact.py) waits for each piece right after its issue.  The
// address is a uniform SGPR base plus a fixed per-lane offset, so a chunk's
// pieces cost no vector arithmetic.
#ifdef WN_DMA_SYNC
#define SMMD_DMA_WAIT "\n\ts_waitcnt vmcnt(0)"
#else
#define SMMD_DMA_WAIT ""
#endif
__device__ __forceinline__ void glds16(uint32_t voff, const void *sbase, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0" SMMD_DMA_WAIT
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds_dst)
                 : "memory");
}

__device__ __forceinline__ void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace smmd

// Shared between the two flash-attention kernels (attention.hip: the 8-wave kernel, its redo and
// the split-tail combine; attention_w4.hip: the 4-wave NC kernel): item geometry, the argument
// block, the item-flag workspace protocol.
#pragma once
#include "common.h"

namespace vs_attn {

constexpr int HD = 128;          // head dim
constexpr int BQ = 256;          // query rows per workgroup (one item)
constexpr int BKV = 64;          // keys per tile
constexpr int PROW = HD + 4;     // split-tail partial row: 128 fp32 O, m, l, 2 pad (16-B aligned)
constexpr float NC_LMIN = 0x1p-64f;
constexpr float NC_LMAX = 0x1p64f;
constexpr float W4_LMIN = 0x1p-4f;   // attn_fwd_w4's lower row-sum bound (attention_w4.hip)

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
    // raw buffer descriptor; out-of-range loads return 0 (rows past Skv, masked anyway)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// Kernel arguments.  The fields an item switch needs (bases, batch strides, nqb, H) are read
// through a volatile view of the argument block at each switch, so they do not stay live in SGPRs
// across the tile loop (they pushed it past the SGPR file).
struct AttnArgs {
    const bf16_t *Q, *K, *V;
    bf16_t* O;
    long long bsq, bsk, bsv, bso;
    long long ldq, ldk, ldv, ldo;
    float* part;
    int* flags;      // item-flag workspace (layout at NcWs): written by the NC kernel / the combine,
                     // consumed and cleared by the redo launch
    float c;
    int Sq, Skv, H, nqb, nmain, npers, nsplit, piece_tiles;
    int nc_cap;      // items the flag workspace holds (its list and its flags)
    unsigned* queue; // attn_fwd_w4's XCD item queues (workspace kind 5 + VS_Q_ATTN words), or null
};

// Item-flag workspace (kind 4, ints; count, done and flags zero between launches): [0] count of
// listed items, [1] redo blocks done reading the count, [2, 2 + cap) one flag per item,
// [2 + cap, 2 + 2 cap) the list of flagged items (an item is listed once: the first flagger's
// atomicExch sees 0).  cap follows from the bound size, so the regions never move.
__device__ __forceinline__ void nc_list_item(int* ws, int cap, int gi) {
    if (atomicExch(ws + 2 + gi, 1) == 0) ws[2 + cap + atomicAdd(ws, 1)] = gi;
}
constexpr int MODE_CHK = 0, MODE_NC = 1, MODE_REDO = 2;

// attn_fwd_w4 launch (attention_w4.hip): grid blocks of 256 threads, 128 KB of dynamic LDS
hipError_t attn_w4_launch(const AttnArgs& args, bool rebase, unsigned grid, hipStream_t stream);

}  // namespace vs_attn

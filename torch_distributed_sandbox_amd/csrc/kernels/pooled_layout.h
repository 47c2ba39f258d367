// Pooled-blocked ("PB") layout of ya [B][32][..], the conv2 output y2 at each 2x2 pooling
// window's argmax (written by the conv2 forward, read by the head forward and backward).  (The
// pooled gradient g2m stays planar, [B][32][Q][Q]: the head backward writes it in the row runs of
// the fc weight it streams.)
//
// Each (image, channel) plane is tiled in blocks of 4 pooled rows x 8 pooled columns, 32
// floats = 128 B per block, blocks row-major:
//
//   index(b, c, py, px) = (((b*32 + c)*Q4 + py/4)*Q8 + px/8)*32 + (py%4)*8 + px%8
//   Q4 = ceil(Q/4), Q8 = ceil(Q/8)
//
// Why: one conv2 output tile (8 x 16 pixels, conv2_fwd2.hip) pools to exactly one block, so the
// forward writes ya as one full 128-B line per channel (a planar ya would be 32-B row pieces);
// and a (channel, block row) of ya is one contiguous run of Q8 blocks, which the head streams
// beside the fc weight's row runs (head_pb.hip).  Entries of a block outside the Q x Q image are
// padding: the producer writes don't-care values, consumers mask them.
#pragma once

#include <stdint.h>

namespace tds {

struct PBGeom {
  int Q, Q4, Q8;
  __host__ __device__ int64_t plane() const { return (int64_t)Q4 * Q8 * 32; }  // floats per (b, c)
  __host__ __device__ int64_t index(int b, int c, int py, int px) const {
    return ((((int64_t)b * 32 + c) * Q4 + (py >> 2)) * Q8 + (px >> 3)) * 32 + (py & 3) * 8 + (px & 7);
  }
};

__host__ __device__ inline PBGeom pb_geom(int Q) { return PBGeom{Q, (Q + 3) / 4, (Q + 7) / 8}; }

}  // namespace tds

// Pooled-blocked ("PB") layout of ya [B][32][..], the conv2 output y2 at each 2x2 pooling
// window's argmax (written by the conv2 forward, read by the head forward and backward), and its
// row-shifted form for the pooled gradient g2m (written by the head backward, read by the conv2
// backward's staging: G2MGeom below).
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

// g2m: the same 4 x 8 blocks with the row blocking shifted by one -- block row R holds pooled rows
// 4R - 3 .. 4R (R = (py + 3) / 4) -- because the conv2 backward stages a tile's NEW rows 8 tr + 2 ..
// 8 tr + 9, whose pooling windows are pooled rows 4 tr + 1 .. 4 tr + 4: exactly block row tr + 1.  A
// tile's pooled gradient per channel is then one 128-B line (its 8 pooled columns) and two halo
// columns from the blocks beside it (3 lines), where the planar layout gave every (channel, pooled
// row) run of 10 floats a line of its own (r6: the texture path costs ~2 cycles per distinct line a
// load instruction touches, profiles/micro/r6_s3_ta_pattern.txt).
//
//   index(b, c, py, px) = (((b*32 + c)*NR + (py+3)/4)*Q8 + px/8)*32 + ((py+3)%4)*8 + px%8
//   NR = (Q+2)/4 + 1, Q8 = ceil(Q/8)
//
// The head backward writes rows < Q (columns past Q of a block as 0); slots of rows >= Q are never
// written and never read unmasked (the conv2 backward's border tiles mask unpooled windows).
struct G2MGeom {
  int Q, NR, Q8;
  __host__ __device__ int64_t plane() const { return (int64_t)NR * Q8 * 32; }  // floats per (b, c)
  __host__ __device__ int64_t index(int b, int c, int py, int px) const {
    return ((((int64_t)b * 32 + c) * NR + ((py + 3) >> 2)) * Q8 + (px >> 3)) * 32 + ((py + 3) & 3) * 8 + (px & 7);
  }
};

__host__ __device__ inline G2MGeom g2m_geom(int Q) { return G2MGeom{Q, (Q + 2) / 4 + 1, (Q + 7) / 8}; }

}  // namespace tds

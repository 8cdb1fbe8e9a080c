// One-wave-per-SIMD attention forward (attn_fwd4.hip): parameters and launcher, called by attn_fwd.hip's
// dispatch for head_dim 64 with the bounded softmax and no document mask.
#pragma once
#include "attn_common.hpp"

struct Fwd4P {
  const bf16 *q, *k, *v;
  bf16* o;
  float* lse;               // [B, H, Lq], base 2
  long ldq, ldk, ldv, ldo;  // token row strides (elements)
  long sqb, skb, svb, sob;  // batch strides (elements)
  long Lq, Lkv;
  int H, B;
  float scale_log2;
  MaskP m;                  // causal / window frame mask (no documents, no q_offset)
};

// queries per workgroup (4 waves x 128)
constexpr int FWD4_QTW = 512;

// 0 on success; -1 if the shape is outside the kernel's domain (the caller keeps attn_fwd16_k)
int owlk_fwd4_launch(const Fwd4P& p, hipStream_t s);

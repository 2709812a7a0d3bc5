// Shared between conv3x3_igemm.hip (configuration table, C ABI) and conv_cin3.hip (the kernel): the
// arguments of the split-bf16 MFMA conv of a 1..3-channel input (configurations 42, 43).
#pragma once
#include <hip/hip_runtime.h>

struct Cin3Args {
  const float* x;
  const float* x2;  // images [nsplit, N) read from x2 (the content|style pair of one launch)
  int nsplit;
  const float* wp;  // packed fp32 [cin_pad8][9][cout_pad] (ast_conv3x3_pack_weights_f32)
  const float* bias;
  float* y_pre;
  float* y_act;
  const float* in_mean;  // ImageNet normalisation in the gather (VGG conv_1), or null
  const float* in_std;
  // input-gradient epilogue of ast_conv3x3_dgrad_f32 on y_pre (ConvArgs e_* of conv3x3_igemm.hip)
  const float* e_mask;
  const float* e_add_pre;
  const float* e_add_post;
  int N, Cin, H, W, Cout, cout_pad;
  int reflect;  // 0: zero pad, 1: ReflectionPad2d(1)
};

// TH = 16 or 8 output rows per workgroup; AST_E_UNSUPPORTED for Cin > 3
int launch_conv_cin3_x3(const Cin3Args& a, int th, hipStream_t s);

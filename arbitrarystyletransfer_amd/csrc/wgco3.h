// Shared between conv3x3_bwd.hip (wgrad plan, C ABI) and wgrad_co3.hip (the kernels): the weight
// gradient of a 3x3 conv with Cout <= 3 on the split-bf16 MFMA (round 6).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct WgCo3Args {
  const float* x;   // [N][Cin][Hin][Win]: the conv's input before upsample / padding
  const float* dy;  // dY: plane stride dy_plane, row stride dy_pitch, element (0, 0) at dy_off
  float* dw;        // partial slots [slot][Cout][Cin][9]
  float* db;        // partial slots [slot][Cout], or null
  int N, Cin, Hin, Win, Cout, reflect, up;
  int dy_pitch;
  int64_t dy_plane, dy_off;
  int tiles_x, tiles_y, cgroups;  // q tiles over the padded rows x interior columns; 64-channel groups
  int64_t ntiles, tiles_per_block, splits;
};

// the q-tile geometry the plan needs (rows of the padded grid x interior columns)
constexpr int WGCO3_TQH = 4, WGCO3_TQW = 64;
// partial slots of the border-column pass (after the main kernel's splits; reflect / upsample only)
constexpr int WGCO3_BORDER_SLOTS = 8;

// true when the MFMA form applies (Cout <= 3, the upsampled width a multiple of 16)
bool wgrad_co3_supported(int cin, int h_in, int w_in, int cout, int up);
// main kernel (slots [0, splits)) and, for reflect padding, the border-column pass (the next
// WGCO3_BORDER_SLOTS slots)
int launch_wgrad_co3(const WgCo3Args& a, hipStream_t s);

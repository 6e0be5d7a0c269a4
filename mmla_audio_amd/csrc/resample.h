// Rate conversion of the offline pre-conditioning (resample.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

// audioop.ratecv(data, 2, nch, inrate, outrate, None) with inrate / outrate already divided by
// their gcd; in [n_frames][nch] int16, out [n_out][nch] int16
hipError_t ratecv_launch(const int16_t* in, int64_t n_frames, int nch, int inrate, int outrate,
                         int16_t* out, int64_t n_out, hipStream_t s);

// resampy.resample_f (one channel): y[t] for t < n_out from x[n_orig], the float64 time register
// tr[t] and the interpolated filter half-window as (win[i], win[i + 1] - win[i]) pairs, nwin of them
struct SincResampleArgs {
  const float* x;
  int64_t n_orig;
  const double* tr;
  const double* win;   // [nwin][2]
  int64_t nwin;
  int num_table;
  int index_step;
  double scale;
  float* y;
  int64_t n_out;
};
hipError_t sinc_resample_launch(const SincResampleArgs& a, hipStream_t s);

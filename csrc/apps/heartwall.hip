// heartwall-shaped template tracking (Rodinia heartwall: one workgroup per
// tracked sample point of the heart wall; each point's template is correlated
// against every displacement in its search window of the next frame, the
// partial sums staged in shared memory, and the best displacement moves the
// point), plain HIP.  Usage: heartwall <frames> <points>
#include <cmath>

#include "app_common.h"

constexpr int kT = 25;       // template side (pixels)
constexpr int kS = 8;        // search radius: (2*kS+1)^2 displacements
constexpr int kThreads = 256;

__global__ void heartwall_kernel(const float* frame, int fw, int fh, const float* tmpl, int* px, int* py) {
  __shared__ float tl[kT * kT];
  __shared__ float best_v[kThreads];
  __shared__ int best_i[kThreads];
  const int p = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < kT * kT; i += kThreads) tl[i] = tmpl[(size_t)p * kT * kT + i];
  __syncthreads();
  const int cx = px[p], cy = py[p], nd = (2 * kS + 1) * (2 * kS + 1);
  float bv = -1e30f;
  int bi = 0;
  for (int d = t; d < nd; d += kThreads) {  // one displacement per thread
    const int dx = d % (2 * kS + 1) - kS, dy = d / (2 * kS + 1) - kS;
    const int ox = cx + dx - kT / 2, oy = cy + dy - kT / 2;
    float num = 0.f, e = 0.f;
    for (int r = 0; r < kT; ++r) {
      const float* row = frame + (size_t)(oy + r) * fw + ox;
      for (int c = 0; c < kT; ++c) {
        const float f = row[c];
        num += f * tl[r * kT + c];
        e += f * f;
      }
    }
    const float v = num * rsqrtf(e + 1e-6f);
    if (v > bv) {
      bv = v;
      bi = d;
    }
  }
  best_v[t] = bv;
  best_i[t] = bi;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {  // arg-max reduction
    if (t < s && (best_v[t + s] > best_v[t] || (best_v[t + s] == best_v[t] && best_i[t + s] < best_i[t]))) {
      best_v[t] = best_v[t + s];
      best_i[t] = best_i[t + s];
    }
    __syncthreads();
  }
  if (t == 0) {
    px[p] = cx + best_i[0] % (2 * kS + 1) - kS;
    py[p] = cy + best_i[0] / (2 * kS + 1) - kS;
  }
}

int main(int argc, char** argv) {
  const int frames = argc > 1 ? atoi(argv[1]) : 1, np = argc > 2 ? atoi(argv[2]) : 51;
  const int fw = 656, fh = 744;  // test.avi frame size
  std::vector<float> frame((size_t)fw * fh), tmpl((size_t)np * kT * kT);
  std::vector<int> px(np), py(np);
  auto img = [&](int x, int y, int f) {  // smooth moving texture
    return 1.f + std::sin(0.05f * (x + 2 * f)) * std::cos(0.07f * (y - f)) + 0.3f * std::sin(0.011f * x * y);
  };
  for (int i = 0; i < np; ++i) {  // points on an ellipse (the wall), templates cut from frame 0
    px[i] = fw / 2 + (int)(180 * std::cos(6.2831853f * i / np));
    py[i] = fh / 2 + (int)(220 * std::sin(6.2831853f * i / np));
    for (int r = 0; r < kT; ++r)
      for (int c = 0; c < kT; ++c) tmpl[((size_t)i * kT + r) * kT + c] = img(px[i] - kT / 2 + c, py[i] - kT / 2 + r, 0);
  }
  float *d_frame, *d_tmpl;
  int *d_px, *d_py;
  APP_HIP(hipMalloc(&d_frame, frame.size() * 4));
  APP_HIP(hipMalloc(&d_tmpl, tmpl.size() * 4));
  APP_HIP(hipMalloc(&d_px, np * 4));
  APP_HIP(hipMalloc(&d_py, np * 4));
  APP_HIP(hipMemcpy(d_tmpl, tmpl.data(), tmpl.size() * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_px, px.data(), np * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_py, py.data(), np * 4, hipMemcpyHostToDevice));
  for (int f = 1; f <= frames; ++f) {
    for (int y = 0; y < fh; ++y)
      for (int x = 0; x < fw; ++x) frame[(size_t)y * fw + x] = img(x, y, 0);  // static scene: points must stay
    APP_HIP(hipMemcpy(d_frame, frame.data(), frame.size() * 4, hipMemcpyHostToDevice));
    heartwall_kernel<<<np, kThreads>>>(d_frame, fw, fh, d_tmpl, d_px, d_py);
    APP_HIP(hipGetLastError());
  }
  std::vector<int> ox(np), oy(np);
  APP_HIP(hipMemcpy(ox.data(), d_px, np * 4, hipMemcpyDeviceToHost));
  APP_HIP(hipMemcpy(oy.data(), d_py, np * 4, hipMemcpyDeviceToHost));
  int moved = 0;
  for (int i = 0; i < np; ++i) moved += (ox[i] != px[i] || oy[i] != py[i]);
  const bool ok = moved <= np / 10;  // a static frame keeps (almost) every point in place
  printf("heartwall frames=%d points=%d: %d moved %s\n", frames, np, moved, ok ? "PASSED" : "FAILED");
  for (void* p : {(void*)d_frame, (void*)d_tmpl, (void*)d_px, (void*)d_py}) APP_HIP(hipFree(p));
  return ok ? 0 : 1;
}

// fp8 (e4m3) conversion probe for the KV-cache path: decodes all 256 codes with
// v_cvt_scalef32_pk_bf16_fp8 at three scales and encodes a float ramp with
// v_cvt_pk_fp8_f32, printing both so the host compares them against
// torch.float8_e4m3fn (bench/probes/fp8_cvt_check.py).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__global__ void dec(unsigned short* out, float s) {
  const unsigned c = threadIdx.x;   // 256 threads, one code each (low byte of the word)
  const unsigned w = c | (c << 8) | (c << 16) | (c << 24);
  const bf16x2_t lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, s, false);
  out[c] = __builtin_bit_cast(unsigned, lo) & 0xffff;
}
__global__ void enc(const float* in, unsigned char* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int p = __builtin_amdgcn_cvt_pk_fp8_f32(in[i], 0.f, 0, false);
  out[i] = (unsigned char)(p & 0xff);
}
int main() {
  unsigned short* d; hipMalloc(&d, 512);
  unsigned short h[256];
  const float scales[3] = {1.f, 0.5f, 3.f};
  for (float s : scales) {
    dec<<<1, 256>>>(d, s);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("dec %g", s);
    for (int i = 0; i < 256; ++i) printf(" %u", h[i]);
    printf("\n");
  }
  const int n = 2001;
  float hin[n];
  for (int i = 0; i < n; ++i) hin[i] = -500.f + 0.5f * i;
  float* din; unsigned char* dout; unsigned char hout[n];
  hipMalloc(&din, n * 4); hipMalloc(&dout, n);
  hipMemcpy(din, hin, n * 4, hipMemcpyHostToDevice);
  enc<<<(n + 255) / 256, 256>>>(din, dout, n);
  hipMemcpy(hout, dout, n, hipMemcpyDeviceToHost);
  printf("enc");
  for (int i = 0; i < n; ++i) printf(" %u", hout[i]);
  printf("\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

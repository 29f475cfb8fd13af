// Probe: f32-input MFMA (v_mfma_f32_16x16x4f32) result layout and sustained
// rate on gfx950 (input to the fp32 path of k_dist_topk).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// A[16][4], B[4][16]; lane l supplies A[l&15][l>>4], B[l>>4][l&15]; dump D registers.
__global__ void layout(const float* A, const float* B, float* D){
  int l = threadIdx.x;
  f4 acc = {0,0,0,0};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(l&15)*4 + (l>>4)], B[(l>>4)*16 + (l&15)], acc, 0,0,0);
  for(int r=0;r<4;r++) D[l*4+r]=acc[r];
}
__global__ void rate(float* out, long long* clk, int iters, float x){
  f4 acc[8];
  for(int i=0;i<8;i++) acc[i] = (f4){0,0,0,0};
  float a = x + threadIdx.x * 0.37f, b = x - threadIdx.x * 0.11f;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for(int it=0; it<iters; it++){
#pragma unroll
    for(int i=0;i<8;i++) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0,0,0);
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s=0; for(int i=0;i<8;i++) s += acc[i][0]+acc[i][1]+acc[i][2]+acc[i][3];
  out[blockIdx.x*blockDim.x+threadIdx.x]=s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
int main(){
  std::vector<float> A(64),B(64),D(256);
  for(int i=0;i<16;i++)for(int k=0;k<4;k++) A[i*4+k] = (float)((i*4+k)%7 - 3);
  for(int k=0;k<4;k++)for(int j=0;j<16;j++) B[k*16+j] = (float)(10*k + j);
  float *dA,*dB,*dD; CK(hipMalloc(&dA,256));CK(hipMalloc(&dB,256));CK(hipMalloc(&dD,1024));
  CK(hipMemcpy(dA,A.data(),256,hipMemcpyHostToDevice));CK(hipMemcpy(dB,B.data(),256,hipMemcpyHostToDevice));
  layout<<<1,64>>>(dA,dB,dD); CK(hipDeviceSynchronize());
  CK(hipMemcpy(D.data(),dD,1024,hipMemcpyDeviceToHost));
  int bad_g=0, bad_f=0;
  for(int l=0;l<64;l++)for(int r=0;r<4;r++){
    int col=l&15, row_g=(l>>4)+4*r, row_f=(l>>4)*4+r;
    float ref_g=0, ref_f=0;
    for(int k=0;k<4;k++){ ref_g += A[row_g*4+k]*B[k*16+col]; ref_f += A[row_f*4+k]*B[k*16+col]; }
    bad_g += D[l*4+r]!=ref_g; bad_f += D[l*4+r]!=ref_f;
  }
  printf("f32 16x16x4 D layout: row=(l>>4)+4r mismatches %d ; row=4(l>>4)+r mismatches %d\n", bad_g, bad_f);
  int nb = 256*4, nt = 256, iters = 100000;
  float* o; long long* clk; CK(hipMalloc(&o,(size_t)nb*nt*4)); CK(hipMalloc(&clk, nb*16));
  hipEvent_t e0,e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  rate<<<nb,nt>>>(o,clk,1000,1.0f);
  CK(hipEventRecord(e0)); rate<<<nb,nt>>>(o,clk,iters,1.0f); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms,e0,e1));
  std::vector<long long> h(nb*2); CK(hipMemcpy(h.data(), clk, nb*16, hipMemcpyDeviceToHost));
  double f=0; for(int b=0;b<nb;b++) f += (double)h[2*b]/h[2*b+1]*100.0; f/=nb;
  double fl = (double)nb*(nt/64)*iters*8*2048.0;
  printf("sustained mfma_f32_16x16x4: %.1f ms %.2f TFLOP/s, in-kernel clock %.0f MHz\n", ms, fl/ms/1e9, f);
  return 0;
}

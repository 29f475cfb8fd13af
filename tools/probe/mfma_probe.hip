// Probe: f64 MFMA fragment layout, f64 MFMA issue rate, global_load_lds lane layout on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// A[16][4], B[4][16]; lane l supplies A[l&15][l>>4], B[l>>4][l&15] (guide §3); dump D registers.
__global__ void layout(const double* A, const double* B, double* D){
  int l = threadIdx.x;
  d4 acc = {0,0,0,0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l&15)*4 + (l>>4)], B[(l>>4)*16 + (l&15)], acc, 0,0,0);
  for(int r=0;r<4;r++) D[l*4+r]=acc[r];
}
template<int NACC>
__global__ void rate(double* out, int iters, double x){
  d4 acc[NACC];
  for(int i=0;i<NACC;i++) acc[i] = (d4){0,0,0,0};
  double a = x + threadIdx.x, b = x - threadIdx.x;
  for(int it=0; it<iters; it++){
#pragma unroll
    for(int i=0;i<NACC;i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0,0,0);
  }
  double s=0; for(int i=0;i<NACC;i++) s += acc[i][0]+acc[i][1]+acc[i][2]+acc[i][3];
  out[blockIdx.x*blockDim.x+threadIdx.x]=s;
}
__global__ void vfma(double* out, int iters, double x){
  double a0=x+threadIdx.x, a1=a0+1,a2=a0+2,a3=a0+3,a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7, b=x*0.5;
  for(int it=0; it<iters; it++){
    a0=fma(a0,b,x);a1=fma(a1,b,x);a2=fma(a2,b,x);a3=fma(a3,b,x);a4=fma(a4,b,x);a5=fma(a5,b,x);a6=fma(a6,b,x);a7=fma(a7,b,x);
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=a0+a1+a2+a3+a4+a5+a6+a7;
}
__global__ void glds(const double* src, double* out){
  __shared__ double s[128];
  int l = threadIdx.x;
  // lane l loads 16 B from src + perm(l)*2 doubles
  int p = (l*7)&63;
  __builtin_amdgcn_global_load_lds((const void*)(src + p*2), (__attribute__((address_space(3))) void*)s, 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  out[l*2] = s[l*2]; out[l*2+1]=s[l*2+1];
}
int main(){
  // layout
  std::vector<double> A(64),B(64),D(256);
  for(int i=0;i<16;i++)for(int k=0;k<4;k++) A[i*4+k] = (i==k)?1.0:0.0; // A = [I4;0] partial identity on first 4 rows
  for(int k=0;k<4;k++)for(int j=0;j<16;j++) B[k*16+j] = 100*k + j;   // asymmetric
  // also full test: A random ints
  for(int i=0;i<16;i++)for(int k=0;k<4;k++) A[i*4+k] = (i*4+k)%7 - 3;
  double *dA,*dB,*dD; CK(hipMalloc(&dA,64*8));CK(hipMalloc(&dB,64*8));CK(hipMalloc(&dD,256*8));
  CK(hipMemcpy(dA,A.data(),512,hipMemcpyHostToDevice));CK(hipMemcpy(dB,B.data(),512,hipMemcpyHostToDevice));
  layout<<<1,64>>>(dA,dB,dD); CK(hipDeviceSynchronize());
  CK(hipMemcpy(D.data(),dD,2048,hipMemcpyDeviceToHost));
  int bad_g=0, bad_f32=0;
  for(int l=0;l<64;l++)for(int r=0;r<4;r++){
    int col=l&15;
    int row_g=(l>>4)+4*r, row_f=(l>>4)*4+r;
    double ref_g=0, ref_f=0;
    for(int k=0;k<4;k++){ ref_g+=A[row_g*4+k]*B[k*16+col]; ref_f+=A[row_f*4+k]*B[k*16+col]; }
    if(ref_g!=D[l*4+r]) bad_g++;
    if(ref_f!=D[l*4+r]) bad_f32++;
  }
  printf("layout: guide-map mismatches=%d  f32-map mismatches=%d\n", bad_g, bad_f32);
  // rate
  int nb=256*8, nt=256, iters=2000; double* o; CK(hipMalloc(&o,(size_t)nb*nt*8));
  hipEvent_t e0,e1; CK(hipEventCreate(&e0));CK(hipEventCreate(&e1));
  for(int rep=0;rep<2;rep++){
    float ms;
    CK(hipEventRecord(e0)); rate<4><<<nb,nt>>>(o,iters,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms,e0,e1));
    double fl = (double)nb*(nt/64)*iters*4*2048.0;
    printf("mfma f64 16x16x4 nacc=4, 1024 thr/CU-ish: %.3f ms  %.2f TFLOP/s\n", ms, fl/ms/1e9);
    CK(hipEventRecord(e0)); rate<8><<<nb,nt>>>(o,iters,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms,e0,e1));
    fl = (double)nb*(nt/64)*iters*8*2048.0;
    printf("mfma f64 nacc=8: %.3f ms  %.2f TFLOP/s\n", ms, fl/ms/1e9);
    CK(hipEventRecord(e0)); rate<1><<<nb,nt>>>(o,iters,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms,e0,e1));
    fl = (double)nb*(nt/64)*iters*1*2048.0;
    printf("mfma f64 nacc=1 (dependent chain): %.3f ms  %.2f TFLOP/s\n", ms, fl/ms/1e9);
    CK(hipEventRecord(e0)); rate<4><<<256,256>>>(o,iters,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms,e0,e1));
    fl = (double)256*(4)*iters*4*2048.0;
    printf("mfma f64 nacc=4, 1 wave/SIMD: %.3f ms  %.2f TFLOP/s\n", ms, fl/ms/1e9);
    CK(hipEventRecord(e0)); vfma<<<nb,nt>>>(o,iters*4,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms,e0,e1));
    fl = (double)nb*nt*iters*4*8*2.0;
    printf("v_fma_f64: %.3f ms  %.2f TFLOP/s\n", ms, fl/ms/1e9);
  }
  // glds
  std::vector<double> S(128), O(128); for(int i=0;i<128;i++) S[i]=i;
  double *dS,*dO; CK(hipMalloc(&dS,1024));CK(hipMalloc(&dO,1024));
  CK(hipMemcpy(dS,S.data(),1024,hipMemcpyHostToDevice));
  glds<<<1,64>>>(dS,dO); CK(hipDeviceSynchronize()); CK(hipMemcpy(O.data(),dO,1024,hipMemcpyDeviceToHost));
  int badl=0; for(int l=0;l<64;l++){ int p=(l*7)&63; if(O[l*2]!=p*2||O[l*2+1]!=p*2+1) badl++; }
  printf("glds lane-linear dest mismatches=%d\n", badl);
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr,0)); printf("dev %s CUs=%d clock=%d kHz\n", pr.gcnArchName, pr.multiProcessorCount, pr.clockRate);
  return 0;
}

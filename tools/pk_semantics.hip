// Probe: do the packed-f32 swizzle/negate forms hipcc emits compute what the
// source says on gfx950?  Compares each kernel against scalar math on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float v2 __attribute__((ext_vector_type(2)));
__global__ void kA(const v2* a, const v2* b, v2* o){ int i=threadIdx.x; v2 x=a[i], y=b[i];
  v2 r = x.xx * y; v2 na = x.yy * v2{-1.f, 1.f}; o[i] = __builtin_elementwise_fma(na, y.yx, r); }
__global__ void kB(const v2* a, const v2* b, v2* o){ int i=threadIdx.x; v2 x=a[i], y=b[i];
  v2 r = x.xx * y; v2 t = x.yy * y.yx; o[i] = r + t * v2{-1.f,1.f}; }
__global__ void kD(const v2* a, const v2* b, v2* o){ int i=threadIdx.x; v2 x=a[i], y=b[i]; v2 r, z;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(x), "v"(y));
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(z) : "v"(x), "v"(y), "v"(r));
  o[i] = z; }
__global__ void kE(const v2* a, const v2* b, v2* o){ int i=threadIdx.x; v2 x=a[i], q=b[i];
  o[i] = x + q.yx*v2{1.f,-1.f}; }
__global__ void kF(const v2* a, const v2* b, v2* o){ int i=threadIdx.x; v2 x=a[i], q=b[i]; v2 z;
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(z) : "v"(x), "v"(q));
  o[i] = z; }
int main(){
  const int n=64; v2 ha[n], hb[n], ho[n];
  for(int i=0;i<n;++i){ ha[i]=(v2)(1.f+i, 0.5f*i-3.f); hb[i]=(v2)(2.f-0.25f*i, 1.f+0.125f*i); }
  v2 *da,*db,*dout; hipMalloc(&da,sizeof ha); hipMalloc(&db,sizeof hb); hipMalloc(&dout,sizeof ho);
  hipMemcpy(da,ha,sizeof ha,hipMemcpyHostToDevice); hipMemcpy(db,hb,sizeof hb,hipMemcpyHostToDevice);
  void (*ks[])(const v2*,const v2*,v2*) = {kA,kB,kD,kE,kF}; const char* names[]={"A cmul vec","B cmul vec","D cmul asm","E p-iq vec","F p-iq asm"};
  int bad_total=0;
  for(int k=0;k<5;++k){ hipLaunchKernelGGL(ks[k], dim3(1), dim3(n), 0, 0, da, db, dout); hipMemcpy(ho,dout,sizeof ho,hipMemcpyDeviceToHost);
    int bad=0; for(int i=0;i<n;++i){ float ex, ey; v2 x=ha[i], y=hb[i];
      if(k<3){ ex=x.x*y.x-x.y*y.y; ey=x.x*y.y+x.y*y.x; } else { ex=x.x+y.y; ey=x.y-y.x; }
      if(fabsf(ho[i].x-ex)>1e-4f*(1+fabsf(ex)) || fabsf(ho[i].y-ey)>1e-4f*(1+fabsf(ey))){ if(!bad) printf("  %s i=%d got (%g,%g) want (%g,%g)\n",names[k],i,ho[i].x,ho[i].y,ex,ey); ++bad; } }
    printf("%s: %s\n", names[k], bad? "WRONG":"ok"); bad_total+=bad; }
  return 0; }

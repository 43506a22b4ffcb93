// Markstein exact-division check (gemm_f32.h div_rn): x * RN(1/d) corrected by one fma residual step
// vs IEEE x / d on random pairs.  gcc -O2 -mfma tools/markstein_check.c -lm && ./a.out 300000000
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static uint64_t s=88172645463325252ULL;
static inline uint64_t nx(){ s^=s<<13; s^=s>>7; s^=s<<17; return s;}
static inline float rf(){ // random float with random exponent in a wide normal range and random sign
  uint32_t m=nx()&0x7fffff; int e=(int)(nx()%60)+127-30; uint32_t sg=(nx()&1)<<31; uint32_t b=sg|((uint32_t)e<<23)|m; float f; memcpy(&f,&b,4); return f;}
int main(int argc,char**argv){
  long n=atol(argv[1]); long bad=0;
  for(long i=0;i<n;i++){
    float x=rf(); float d=fabsf(rf());
    if(i%3==0){ // realistic: d = sqrtf(v+eps) with v in [0.5,1.5]
      float v=0.5f+(float)(nx()%1000000)/1e6f; d=sqrtf(v+1e-5f); }
    float y=1.0f/d;
    float q=x*y;
    float r=fmaf(-q,d,x);
    float q2=fmaf(r,y,q);
    float ref=x/d;
    if(memcmp(&q2,&ref,4)!=0){ if(bad<10) printf("x=%a d=%a ref=%a got=%a\n",x,d,ref,q2); bad++; }
  }
  printf("n=%ld bad=%ld\n",n,bad);
}

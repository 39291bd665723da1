/* Host check of the device div_rn() (factormodeling_amd/csrc/fmx_common.hpp): the
 * reciprocal + two fma corrections quotient must equal the IEEE quotient a / b for the
 * divisors the kernels use (counts 1..64, 210 = the ts_decay(20) weight sum, ...).
 *   gcc -O2 -mfma -o /tmp/div_rn_check tools/div_rn_check.c -lm && /tmp/div_rn_check
 * Prints the number of mismatches after two corrections (bad2, must be 0) and after one
 * (bad1, informational). */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static uint64_t s=88172645463325252ull;
static uint64_t xr(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
static double bits(uint64_t b){ double d; memcpy(&d,&b,8); return d; }
static inline double qdiv(double a, double b, double y){
  double q = a*y;
  double e = fma(-q,b,a); q = fma(e,y,q);
  e = fma(-q,b,a); q = fma(e,y,q);
  return q;
}
static inline double qdiv1(double a, double b, double y){
  double q = a*y;
  double e = fma(-q,b,a); q = fma(e,y,q);
  return q;
}
int main(){
  long bad=0, bad1=0, n=0;
  double bs[80]; int nb=0;
  for(int k=1;k<=64;k++) bs[nb++]=k;
  bs[nb++]=210; bs[nb++]=55; bs[nb++]=1830; bs[nb++]=3;
  /* non-integer divisors (row standard deviations): random significands, exponents +-40 */
  for(int k=0;k<8;k++){ uint64_t r=xr(); bs[nb++]=bits(((uint64_t)(1023-40+(r%80))<<52)|(xr()&((1ull<<52)-1))); }
  for(int bi=0;bi<nb;bi++){
    double b=bs[bi], y=1.0/b;
    for(long i=0;i<5000000;i++){
      uint64_t r=xr();
      // exponents in a moderate range [-900, 900], random mantissa, random sign
      uint64_t e=(uint64_t)(1023-850+(r%1700));
      uint64_t m=xr()&((1ull<<52)-1);
      if(i%4==0) m = (m & ~((1ull<<40)-1)); // fewer mantissa bits (decimal-ish)
      if(i%8==1) m = (1ull<<52)-1-(m&0xff);
      double a=bits(((r>>63)<<63)|(e<<52)|m);
      double t=a/b;
      double q=qdiv(a,b,y), q1=qdiv1(a,b,y);
      if(memcmp(&q,&t,8)) { if(bad<5) printf("bad a=%.17g b=%g got %.17g want %.17g\n",a,b,q,t); bad++; }
      if(memcmp(&q1,&t,8)) bad1++;
      n++;
    }
  }
  printf("n=%ld bad2=%ld bad1=%ld\n",n,bad,bad1);
}

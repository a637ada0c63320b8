// rule_search.c -- exhaustive search: can the tail of the B3/S23 rule (after the two full adders,
// n9 = u0 + 2(k0 + x + 2y)) be computed by THREE v_bitop3 gates instead of four?  Tool, not product code.
//   gcc -O2 scripts/rule_search.c -o /tmp/rs && /tmp/rs
// exhaustive: 3 LUT3 gates computing g(u0,k0,x,y,al) over 5 inputs
#include <stdio.h>
#include <stdint.h>
int main(){
  uint32_t in[5]; // truth tables over 32 rows
  for(int i=0;i<5;i++){in[i]=0;for(int r=0;r<32;r++) if(r>>i&1) in[i]|=1u<<r;}
  uint32_t tgt=0;
  for(int r=0;r<32;r++){int u0=r&1,k0=r>>1&1,x=r>>2&1,y=r>>3&1,al=r>>4&1;int S=k0+x+2*y;int f=u0?(S==1):(al&&S==2); if(f) tgt|=1u<<r;}
  printf("tgt %08x\n",tgt);
  uint32_t sig[8]; for(int i=0;i<5;i++) sig[i]=in[i];
  long found=0;
  // gate1 over 5 inputs
  for(int a=0;a<5;a++)for(int b=a+1;b<5;b++)for(int c=b+1;c<5;c++)for(int t1=0;t1<256;t1++){
    uint32_t g1=0; for(int r=0;r<32;r++){int idx=((sig[a]>>r&1)<<2)|((sig[b]>>r&1)<<1)|(sig[c]>>r&1); if(t1>>idx&1) g1|=1u<<r;}
    sig[5]=g1;
    for(int d=0;d<6;d++)for(int e=d+1;e<6;e++)for(int f=e+1;f<6;f++){ if(f!=5) continue; // gate2 uses g1? try both below
    }
    for(int d=0;d<6;d++)for(int e=d+1;e<6;e++)for(int f=e+1;f<6;f++)for(int t2=0;t2<256;t2++){
      uint32_t g2=0; for(int r=0;r<32;r++){int idx=((sig[d]>>r&1)<<2)|((sig[e]>>r&1)<<1)|(sig[f]>>r&1); if(t2>>idx&1) g2|=1u<<r;}
      sig[6]=g2;
      for(int p=0;p<7;p++)for(int q=p+1;q<7;q++)for(int s=q+1;s<7;s++){
        // consistency: rows with same (p,q,s) must share tgt
        int map[8]; for(int k=0;k<8;k++)map[k]=-1; int ok=1;
        for(int r=0;r<32&&ok;r++){int idx=((sig[p]>>r&1)<<2)|((sig[q]>>r&1)<<1)|(sig[s]>>r&1); int v=tgt>>r&1; if(map[idx]<0)map[idx]=v; else if(map[idx]!=v) ok=0;}
        if(ok){ if(found<10) printf("g1(%d,%d,%d,%02x) g2(%d,%d,%d,%02x) out(%d,%d,%d)\n",a,b,c,t1,d,e,f,t2,p,q,s); found++;}
      }
    }
  }
  printf("found %ld\n",found);
}

/* Config 4 (Erdos-Renyi, 2^24 ids, 16 windows of 2^20 edges, seed 2): per close, the seen vertices, the
 * non-roots a full-pass close tests against the hooked-root bitmap, and the vertices it relabels (members
 * of roots hooked in the window) -- the counts behind DESIGN.md section 8 config-4 record.
 * Test-side analysis (links the oracle generator):
 *   gcc -O2 -I oracle -o /tmp/c4cc tests/c4_close_counts.c oracle/gen.c oracle/disjoint_set.c && /tmp/c4cc */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "oracle.h"
static uint32_t* par;
static uint32_t find(uint32_t x){ while(par[x]!=x){ par[x]=par[par[x]]; x=par[x];} return x; }
int main(){
  const uint64_t V=1ull<<24, W=1ull<<20, NW=16;
  int64_t *s=malloc(8*W), *d=malloc(8*W);
  par=malloc(4*V); uint32_t* lab=malloc(4*V); uint8_t* seen=calloc(V,1);
  for(uint64_t v=0;v<V;++v){par[v]=v;lab[v]=v;}
  for(uint64_t w=0;w<NW;++w){
    gso_gen_er(s,d,w*W,W,V,2);
    uint64_t hooks=0;
    for(uint64_t i=0;i<W;++i){ uint32_t a=s[i],b=d[i]; seen[a]=seen[b]=1; uint32_t ra=find(a),rb=find(b); if(ra!=rb){ if(ra<rb) par[rb]=ra; else par[ra]=rb; ++hooks;} }
    uint64_t ns=0, nonroot=0, relab=0, giant=0; 
    // close: flatten
    for(uint64_t v=0;v<V;++v){ if(!seen[v]) continue; ++ns; if(lab[v]!=v) ++nonroot; uint32_t r=find(v); if(r!=lab[v]) ++relab; lab[v]=r; }
    // largest component
    uint32_t* cnt=calloc(V,4); uint32_t mx=0; for(uint64_t v=0;v<V;++v) if(seen[v]){ uint32_t c=++cnt[lab[v]]; if(c>mx) mx=c;} free(cnt);
    printf("w %2llu seen %8llu nonroot_at_close %8llu relabelled %8llu hooks %7llu largest %8u\n",(unsigned long long)w+1,(unsigned long long)ns,(unsigned long long)nonroot,(unsigned long long)relab,(unsigned long long)hooks,mx);
  }
}

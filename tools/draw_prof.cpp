#include <chrono>
#include <cstdio>
#include <x86intrin.h>
// Developer tool (not part of the library): host sampler microbenchmark on the
// bench workload; build like tools/sampler_prof.cpp.
#include "../graphsage-pytorch_amd/csrc/host/sampler.cpp"
namespace gs {
[[maybe_unused]] static void materialise(const Graph& g, Hop& h, bool gcn) {
    HopScratch sc;
    build_sets(g, h, sc, nullptr);
    union_map(h, sc);
    lists(h, sc, gcn);
}
}  // namespace gs
int main(){
  const int scale=21; const int64_t pairs=20000000; const int64_t n=int64_t(1)<<scale;
  std::vector<int64_t> src(pairs), dst(pairs); int64_t np=0;
  gs_rmat_pairs(scale,pairs,0.57,0.19,0.19,824,1,8,src.data(),dst.data(),&np);
  gs_graph* gp=nullptr; gs_graph_build(src.data(),dst.data(),np,n,8,&gp);
  const auto& g=*reinterpret_cast<const gs::Graph*>(gp);
  std::vector<int64_t> cand; for(int64_t v=0;v<n;++v) if(g.degree(v)>0) cand.push_back(v);
  gs::MT19937 rng; rng.init_genrand(824); uint64_t lcg=12345;
  std::vector<int64_t> roots(512); for(auto&r:roots){lcg=lcg*6364136223846793005ull+1442695040888963407ull; r=cand[(lcg>>33)%cand.size()];}
  gs::Hop h0; h0.k=25; h0.dst_ids=roots; gs::draw_positions(g,rng,h0); gs::materialise(g,h0,false);
  std::vector<int64_t> fr=h0.src_ids; const int64_t* rp=g.row_ptr.data();
  std::vector<int64_t> deg(fr.size()); for(size_t i=0;i<fr.size();++i) deg[i]=rp[fr[i]+1]-rp[fr[i]];
  int32_t out[64]; int32_t pool[128]; const int64_t ss=gs::sample_setsize(10);
  uint64_t tsel=0,tpool=0,nsel=0,npool=0,words=0; int reps=200;
  for(int rep=0;rep<reps;++rep) for(size_t i=0;i<fr.size();++i){ int64_t d=deg[i]; if(d<10) continue;
     int idx0=rng.index; uint64_t a=__rdtsc(); gs::sample_positions(rng,d,10,ss,out,pool); uint64_t b=__rdtsc();
     if(d<=ss){tpool+=b-a;npool++;} else {tsel+=b-a;nsel++;} }
  auto a=std::chrono::steady_clock::now(); uint64_t c0=__rdtsc(); for(int i=0;i<100000;i++) rng.twist(); uint64_t c1=__rdtsc();
  auto b=std::chrono::steady_clock::now(); double ns=std::chrono::duration<double,std::nano>(b-a).count();
  double cyc_per_ns=(c1-c0)/ns;
  printf("tsc GHz %.2f; select %.1f ns/call (%lu); pool %.1f ns/call (%lu); twist %.1f ns/block\n",cyc_per_ns,tsel/cyc_per_ns/nsel,nsel,tpool/cyc_per_ns/npool,npool, ns/100000);
}

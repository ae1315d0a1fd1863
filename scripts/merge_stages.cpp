// Host-tail stage timing over the Src10 +-180 candidate records (tests/golden/merge_src10_180.npz -> .bin):
// the same steps as merge_candidates (fpm_engine.hip) with a clock around each.  Profiling aid, not a test.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../fastest_image_pattern_matching_amd/csrc/fpm_host.h"
#include "../include/fpm.h"
#ifdef FPM_HOST_STATS
namespace fpm { extern long g_stats[40]; }
#endif
using namespace fpm;
static double now(){return std::chrono::duration<double,std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();}
int main(int argc,char**argv){
  FILE*f=fopen(argc>1?argv[1]:"/tmp/src10_cands.bin","rb"); std::vector<fpm_candidate> c(10000); int n=fread(c.data(),sizeof(fpm_candidate),10000,f); fclose(f);
  const double D2R=3.1415926535897932384626433832795/180.0;
  for(int it=0;it<20;++it){
  double t0=now();
  struct Key{double s;int i;}; std::vector<Key> o(n); for(int i=0;i<n;++i)o[i]={c[i].top_score,i};
  std::sort(o.begin(),o.end(),[](const Key&a,const Key&b){return a.s>b.s;});
  std::vector<HostMatch> all; for(auto&k:o){auto&x=c[k.i]; if(!x.kept)continue; HostMatch m{}; m.ptx=x.x;m.pty=x.y;m.score=x.score;m.angle=x.angle; all.push_back(m);}
  double t1=now();
  filter_with_score(all,0.7);
  double t2=now();
  for(auto&m:all){double rad=-m.angle*D2R; F2 lt=f2((float)m.ptx,(float)m.pty); F2 rt=f2(lt.x+54*(float)std::cos(rad),lt.y-54*(float)std::sin(rad)); F2 rb=f2(rt.x+54*(float)std::sin(rad),rt.y+54*(float)std::cos(rad)); m.rect=rrect_from3(lt,rt,rb); m.del=false;}
  double t3=now();
  filter_with_rotated_rect(all,0.0);
  double t4=now();
  std::sort(all.begin(),all.end(),score_big2small);
  double t5=now();
  printf("n=%d sort+collect %.3f score %.3f rects %.3f rotrect %.3f final %.3f -> %zu\n",n,t1-t0,t2-t1,t3-t2,t4-t3,t5-t4,all.size());
  }
#ifdef FPM_HOST_STATS
  for(int k=0;k<40;++k) if(fpm::g_stats[k]) printf("stat %d: %ld\n",k,fpm::g_stats[k]/20);
#endif
}

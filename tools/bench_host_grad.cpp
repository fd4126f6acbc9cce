#include <chrono>
#include <cstdio>
#include <vector>
#include <cstdint>
extern "C" int svgd_model_create(void **out, int dim, int ncomp, const double *mus, const double *covs);
extern "C" int svgd_model_logp_grad(void *model, const double *X, int64_t nrows, double *G);
int main(){
  const int d=64; const long n=65536;
  std::vector<double> X(n*d), G(n*d), mu(d,0.0), cov(d*d,0.0);
  for (int r=0;r<d;++r) cov[r*d+r]=1.0;
  for (long e=0;e<n*d;++e) X[e]=(double)((e*2654435761u)%1000)/500.0-1.0;
  void* m; svgd_model_create(&m,d,1,mu.data(),cov.data());
  for(int it=0;it<3;++it){ auto t=std::chrono::steady_clock::now(); svgd_model_logp_grad(m,X.data(),n,G.data());
  printf("%.2f ms\n", std::chrono::duration<double,std::milli>(std::chrono::steady_clock::now()-t).count()); }
}

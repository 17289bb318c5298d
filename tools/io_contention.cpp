// tools/io_contention.cpp — build: g++ -O2 -pthread tools/io_contention.cpp -o build/bin/io_contention
// Concurrent small-file rewrite cost on tmpfs: T threads of one process vs T processes.
// Each pair = open(existing, O_WRONLY) + pwritev(12 KB) + close, twice; also a load-like read
// (open + pread 131 KB + close). CPU time per op from thread/process CPU clocks.
#include <fcntl.h>
#include <sys/uio.h>
#include <sys/wait.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <unistd.h>
#include <sys/stat.h>
#include <sched.h>
#include <linux/capability.h>
#include <sys/syscall.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <time.h>
static double now(){return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();}
static long long tcpu(){timespec t;clock_gettime(CLOCK_THREAD_CPUTIME_ID,&t);return t.tv_sec*1000000000LL+t.tv_nsec;}
int main(int argc,char**argv){
  if(argc<6){fprintf(stderr,"usage: io_contention root T nfiles reps mode(0 threads|1 procs|2 threads+unshare files|3 +fs|4 unshare files+private cred) [mmap]\n");return 2;}
  const bool use_mmap = argc > 6 && atoi(argv[6]) != 0;  // loads: mmap(MAP_POPULATE) + sum + munmap instead of pread
  const char* root=argv[1]; int T=atoi(argv[2]); int nfiles=atoi(argv[3]); int reps=atoi(argv[4]); int procs=atoi(argv[5]);
  const size_t seg=12000, rsz=131*1024;
  std::vector<uint8_t> src((size_t)nfiles*seg*2+4096); for(size_t i=0;i<src.size();++i) src[i]=(uint8_t)(i*131);
  int nd=20; for(int d=0;d<nd;++d){ std::string p=std::string(root)+"/d"+std::to_string(d); mkdir(p.c_str(),0755);}
  std::vector<int> dfd(nd); for(int d=0;d<nd;++d) dfd[d]=open((std::string(root)+"/d"+std::to_string(d)).c_str(),O_PATH|O_DIRECTORY);
  auto name=[&](int i,int k){return "f"+std::to_string(i)+(k==0?"_o.jpg":k==1?"_p.jpg":".dcm");};
  std::vector<uint8_t> big(rsz,7);
  for(int i=0;i<nfiles;++i){ for(int k=0;k<2;++k){int fd=openat(dfd[i%nd],name(i,k).c_str(),O_WRONLY|O_CREAT,0644); if(write(fd,src.data(),seg)<0) return 3; close(fd);}
    int fd=openat(dfd[i%nd],name(i,2).c_str(),O_WRONLY|O_CREAT,0644); if(write(fd,big.data(),rsz)<0) return 3; close(fd);}
  auto* shared=(std::atomic<long long>*)mmap(nullptr,4096,PROT_READ|PROT_WRITE,MAP_SHARED|MAP_ANONYMOUS,-1,0);
  for(int r=0;r<reps;++r){
    new(&shared[0]) std::atomic<long long>(0); new(&shared[1]) std::atomic<long long>(0); new(&shared[2]) std::atomic<long long>(0);
    auto work=[&](int t){ std::vector<uint8_t> buf(rsz); long long cw=0, cr=0;
      std::vector<int> my=dfd;
      if(procs==4){  // private struct cred: capset(current caps) commits a fresh cred for this thread only,
        // so every open/close's get_cred/put_cred (file->f_cred) hits a per-thread refcount line
        __user_cap_header_struct h{_LINUX_CAPABILITY_VERSION_3, 0}; __user_cap_data_struct c[2]{};
        if(syscall(SYS_capget,&h,c)!=0||syscall(SYS_capset,&h,c)!=0) abort(); }
      if(procs==2||procs==3||procs==4){ if(unshare(procs==3?(CLONE_FILES|CLONE_FS):CLONE_FILES)!=0) abort();  // private fd table (+fs_struct)
        for(int d=0;d<nd;++d) my[d]=open((std::string(root)+"/d"+std::to_string(d)).c_str(),O_PATH|O_DIRECTORY); }
      for(int i=t;i<nfiles;i+=T){
        long long c0=tcpu();
        int fd=openat(my[i%nd],name(i,2).c_str(),O_RDONLY);
        if(use_mmap){ void* m=mmap(nullptr,rsz,PROT_READ,MAP_PRIVATE|MAP_POPULATE,fd,0); if(m==MAP_FAILED) abort();
          const uint64_t* q=(const uint64_t*)m; uint64_t acc=0; for(size_t k=0;k<rsz/8;k+=8) acc+=q[k]; buf[0]=(uint8_t)acc; munmap(m,rsz); }
        else if(pread(fd,buf.data(),rsz,0)<0) abort();
        close(fd);
        long long c1=tcpu(); cr+=c1-c0;
        for(int k=0;k<2;++k){ const uint8_t* s=src.data()+((size_t)i*2+k)*seg;
          int f2=openat(my[i%nd],name(i,k).c_str(),O_WRONLY); iovec v[1]={{(void*)s,seg}}; if(pwritev(f2,v,1,0)<0) abort(); close(f2);}
        cw+=tcpu()-c1; }
      shared[0]+=cr; shared[1]+=cw; };
    double t0=now();
    if(procs==1){ std::vector<pid_t> ps; for(int t=0;t<T;++t){pid_t p=fork(); if(p==0){work(t); _exit(0);} ps.push_back(p);} for(auto p:ps) waitpid(p,nullptr,0); }
    else { std::vector<std::thread> th; for(int t=0;t<T;++t) th.emplace_back(work,t); for(auto&x:th) x.join(); }
    double dt=now()-t0;
    printf("T=%2d %s%s  read %.2f us/file  write %.2f us/pair  wall %.1f ms\n",T,procs==1?"procs  ":procs==2?"unshare":procs==3?"unsh+fs":procs==4?"unsh+cr":"threads",use_mmap?"+mmap":"",shared[0].load()/1e3/nfiles,shared[1].load()/1e3/nfiles,dt*1e3);
  }
}

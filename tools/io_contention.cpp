// tools/io_contention.cpp — build: g++ -O2 -pthread tools/io_contention.cpp -o build/bin/io_contention
// Concurrent small-file rewrite cost on tmpfs: T threads of one process vs T processes.
// Each pair = open(existing, O_WRONLY) + pwritev(12 KB) + close, twice; also a load-like read
// (open + pread 131 KB + close). CPU time per op from thread/process CPU clocks. Mode 5: the same
// operations as linked io_uring chains (open into a direct descriptor → read/write → close), a batch
// of files per submit, private fd tables; its CPU is the process's (io-wq workers included).
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
#include <linux/io_uring.h>
#include <sys/resource.h>

// Minimal io_uring (raw syscalls; no liburing in the image).
struct Ring {
  int fd = -1;
  unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
  io_uring_sqe* sqes;
  io_uring_cqe* cqes;
  unsigned pending = 0;
  bool init(unsigned entries, int nfixed) {
    io_uring_params p{};
    fd = (int)syscall(__NR_io_uring_setup, entries, &p);
    if (fd < 0) return false;
    size_t sql = p.sq_off.array + p.sq_entries * sizeof(unsigned), cql = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    size_t l = sql > cql ? sql : cql;
    auto* q = (char*)mmap(nullptr, l, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQ_RING);
    sqes = (io_uring_sqe*)mmap(nullptr, p.sq_entries * sizeof(io_uring_sqe), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQES);
    if (q == MAP_FAILED || sqes == MAP_FAILED) return false;
    sq_head = (unsigned*)(q + p.sq_off.head); sq_tail = (unsigned*)(q + p.sq_off.tail); sq_mask = (unsigned*)(q + p.sq_off.ring_mask);
    sq_array = (unsigned*)(q + p.sq_off.array);
    cq_head = (unsigned*)(q + p.cq_off.head); cq_tail = (unsigned*)(q + p.cq_off.tail); cq_mask = (unsigned*)(q + p.cq_off.ring_mask);
    cqes = (io_uring_cqe*)(q + p.cq_off.cqes);
    std::vector<int> fds(nfixed, -1);
    return syscall(__NR_io_uring_register, fd, IORING_REGISTER_FILES, fds.data(), nfixed) == 0;
  }
  io_uring_sqe* get() {
    unsigned t = *sq_tail, i = t & *sq_mask;
    io_uring_sqe* e = &sqes[i];
    memset(e, 0, sizeof(*e));
    sq_array[i] = i;
    __atomic_store_n(sq_tail, t + 1, __ATOMIC_RELEASE);
    ++pending;
    return e;
  }
  // Submits everything queued and waits for all of it; aborts on a failed op.
  void run() {
    unsigned n = pending; pending = 0;
    if (syscall(__NR_io_uring_enter, fd, n, n, IORING_ENTER_GETEVENTS, nullptr, 0) < 0) abort();
    unsigned got = 0;
    while (got < n) {
      unsigned h = *cq_head, t = __atomic_load_n(cq_tail, __ATOMIC_ACQUIRE);
      if (h == t) { if (syscall(__NR_io_uring_enter, fd, 0, n - got, IORING_ENTER_GETEVENTS, nullptr, 0) < 0) abort(); continue; }
      for (; h != t; ++h, ++got) if (cqes[h & *cq_mask].res < 0) { fprintf(stderr, "io_uring op failed: %d\n", cqes[h & *cq_mask].res); abort(); }
      __atomic_store_n(cq_head, h, __ATOMIC_RELEASE);
    }
  }
};
static double now(){return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();}
static long long tcpu(){timespec t;clock_gettime(CLOCK_THREAD_CPUTIME_ID,&t);return t.tv_sec*1000000000LL+t.tv_nsec;}
int main(int argc,char**argv){
  if(argc<6){fprintf(stderr,"usage: io_contention root T nfiles reps mode(0 threads|1 procs|2 threads+unshare files|3 +fs|4 unshare files+private cred|5 unshare files+io_uring) [mmap|batch]\n");return 2;}
  const bool use_mmap = argc > 6 && atoi(argv[6]) != 0 && atoi(argv[5]) != 5;
  const int batch = argc > 6 && atoi(argv[5]) == 5 ? atoi(argv[6]) : 8;  // mode 5: files per submit  // loads: mmap(MAP_POPULATE) + sum + munmap instead of pread
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
      if(procs==5){ if(unshare(CLONE_FILES)!=0) abort();
        for(int d=0;d<nd;++d) my[d]=open((std::string(root)+"/d"+std::to_string(d)).c_str(),O_PATH|O_DIRECTORY);
        Ring ring; if(!ring.init(4*batch*4, 3*batch)) { fprintf(stderr,"io_uring unavailable\n"); abort(); }
        std::vector<std::string> names((size_t)3*batch); std::vector<uint8_t> rb((size_t)batch*rsz);
        std::vector<int> mine; for(int i=t;i<nfiles;i+=T) mine.push_back(i);
        for(size_t b0=0;b0<mine.size();b0+=batch){
          size_t nb=std::min<size_t>(batch,mine.size()-b0);
          for(size_t j=0;j<nb;++j){ int i=mine[b0+j];
            for(int k=0;k<3;++k){ names[3*j+k]=name(i,k); unsigned slot=(unsigned)(3*j+k);
              io_uring_sqe* e=ring.get(); e->opcode=IORING_OP_OPENAT; e->fd=my[i%nd]; e->addr=(uint64_t)names[3*j+k].c_str();
              e->open_flags=k==2?O_RDONLY:O_WRONLY; e->file_index=slot+1; e->flags=IOSQE_IO_LINK;
              e=ring.get(); e->opcode=k==2?IORING_OP_READ:IORING_OP_WRITE; e->fd=(int)slot; e->flags=IOSQE_FIXED_FILE|IOSQE_IO_LINK;
              if(k==2){ e->addr=(uint64_t)(rb.data()+j*rsz); e->len=(unsigned)rsz; }
              else { e->addr=(uint64_t)(src.data()+((size_t)i*2+k)*seg); e->len=(unsigned)seg; }
              e=ring.get(); e->opcode=IORING_OP_CLOSE; e->file_index=slot+1; } }
          ring.run(); }
        return; }
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
    double t0=now(); rusage ru0; getrusage(RUSAGE_SELF,&ru0);
    if(procs==1){ std::vector<pid_t> ps; for(int t=0;t<T;++t){pid_t p=fork(); if(p==0){work(t); _exit(0);} ps.push_back(p);} for(auto p:ps) waitpid(p,nullptr,0); }
    else { std::vector<std::thread> th; for(int t=0;t<T;++t) th.emplace_back(work,t); for(auto&x:th) x.join(); }
    double dt=now()-t0; rusage ru1; getrusage(procs==1?RUSAGE_CHILDREN:RUSAGE_SELF,&ru1);
    if(procs==1) ru0=rusage{};  // children: cumulative over reps; report the last rep's share below
    auto us=[](const rusage& r){return (r.ru_utime.tv_sec+r.ru_stime.tv_sec)*1e6+r.ru_utime.tv_usec+r.ru_stime.tv_usec;};
    double pcpu=(us(ru1)-us(ru0))/nfiles; if(procs==1) pcpu/=(r+1);
    printf("T=%2d %s%s  read %.2f us/file  write %.2f us/pair  process %.2f us/file+pair  wall %.1f ms\n",T,procs==1?"procs  ":procs==2?"unshare":procs==3?"unsh+fs":procs==4?"unsh+cr":procs==5?"uring  ":"threads",use_mmap?"+mmap":"",shared[0].load()/1e3/nfiles,shared[1].load()/1e3/nfiles,pcpu,dt*1e3);
  }
}

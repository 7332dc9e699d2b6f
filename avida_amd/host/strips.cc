// avgpu_strips -- the C++ host driver of strip-tiled worlds over the C-ABI.
//
// The compiled counterpart of avida_amd/tiles.py (StripWorld) and of bench.py's
// world setup: one 1024 x (1024 N) torus (configs[2] per GPU) cut into row
// strips, one strip per rank, the strips' per-update exchanges done with RCCL
// on the world's own HIP stream (no host synchronisation inside an update), or
// T strips of one process on one GPU exchanging by device copies (loopback,
// the single-GPU check of the protocol).  It replaces what the reference's
// cMultiProcessWorld does between processes (main/cMultiProcessWorld.cc:142-190
// migrants, :375-405 update size) with strips of ONE torus, so the T-strip
// world is the untiled world cell for cell.
//
//   avgpu_strips --config DIR [--side 1024] [--strips T] [--updates U]
//                [--burn-in B] [--seed S] [--gpus N] [--untiled] [--rccl] [--independent]
//
// --independent: every rank runs a whole side x side world of its own and the
// ranks share only the scheduler's update size -- cMultiProcessWorld's
// MP_SCHEDULING (main/cMultiProcessWorld.cc:375-405): avgpu_update_totals, an
// RCCL all-reduce of {sum merit, organisms} on the world's stream,
// avgpu_update_run.  With one rank it is the untiled world.
//
// DIR holds the world's inputs in the reference's formats: instset-classic.cfg
// (legacy "name redundancy" lines or INST lines), environment-logic9.cfg
// (REACTION lines on logic-9 tasks) and detail-50000.pop (the evolved
// genotypes every cell is filled from, cell c taking genotype
// (c * 2654435761) mod pool, bench.py _genomes_for).  Multi-rank: run under
// torch.distributed.run / mpirun-style env (RANK, WORLD_SIZE, LOCAL_RANK,
// MASTER_PORT) or let --gpus N start the N ranks itself.  Prints one JSON line
// (rank 0): updates/s, organism-instructions/s and a digest of every cell's
// state (avgpu_state_digests) over the whole torus.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "avida_gpu.h"

namespace {

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) die(std::string(#x) + ": " + hipGetErrorString(e_)); } while (0)
#define NCCL_OK(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) die(std::string(#x) + ": " + ncclGetErrorString(r_)); } while (0)
#define AV_OK(x) do { if ((x) < 0) die(std::string(#x) + ": " + avgpu_last_error()); } while (0)

[[noreturn]] void die(const std::string& msg) {
  fprintf(stderr, "avgpu_strips: %s\n", msg.c_str());
  exit(2);
}

std::vector<std::string> lines_of(const std::string& path) {
  std::ifstream f(path);
  if (!f) die("cannot read " + path);
  std::vector<std::string> out;
  std::string l;
  while (std::getline(f, l)) out.push_back(l);
  return out;
}

std::vector<std::string> words(const std::string& l) {
  std::istringstream s(l);
  std::vector<std::string> w;
  std::string x;
  while (s >> x) {
    if (x[0] == '#') break;
    w.push_back(x);
  }
  return w;
}

// ---- instruction set: cInstSet::Load (cpu/cInstSet.cc:152-312) for the 26
// heads_default instructions; legacy lines "name redundancy ..." or INST lines
struct InstSet {
  std::vector<uint8_t> handler;
  std::vector<int32_t> redundancy;
};

InstSet read_instset(const std::string& path) {
  static const char* names[AVGPU_H_COUNT] = {
      "nop-A", "nop-B", "nop-C", "if-n-equ", "if-less", "pop", "push", "swap-stk", "swap",
      "shift-r", "shift-l", "inc", "dec", "add", "sub", "nand", "IO", "h-alloc", "h-divide",
      "h-copy", "h-search", "mov-head", "jmp-head", "get-head", "if-label", "set-flow"};
  std::map<std::string, int> id;
  for (int k = 0; k < AVGPU_H_COUNT; k++) id[names[k]] = k;
  InstSet is;
  for (const std::string& l : lines_of(path)) {
    std::vector<std::string> w = words(l);
    if (w.empty()) continue;
    std::string name;
    int red = 1;
    if (w[0] == "INST") {
      if (w.size() < 2) continue;
      name = w[1];
      for (size_t k = 2; k < w.size(); k++)
        if (w[k].rfind("redundancy=", 0) == 0) red = atoi(w[k].c_str() + 11);
    } else if (w[0].find(':') != std::string::npos || w[0] == "INSTSET") {
      continue;
    } else {
      name = w[0];
      if (w.size() > 1) red = atoi(w[1].c_str());
    }
    auto it = id.find(name);
    if (it == id.end()) die("instruction outside heads_default: " + name);
    is.handler.push_back((uint8_t)it->second);
    is.redundancy.push_back(red);
  }
  return is;
}

// ---- environment: REACTION lines on logic-9 tasks (main/cEnvironment.cc:1185-1211)
std::vector<avgpu_reaction> read_environment(const std::string& path) {
  static const std::map<std::string, int> task = {
      {"not", AVGPU_T_NOT}, {"nand", AVGPU_T_NAND}, {"and", AVGPU_T_AND}, {"orn", AVGPU_T_ORN},
      {"or", AVGPU_T_OR}, {"andn", AVGPU_T_ANDN}, {"nor", AVGPU_T_NOR}, {"xor", AVGPU_T_XOR},
      {"equ", AVGPU_T_EQU}};
  std::vector<avgpu_reaction> out;
  for (const std::string& l : lines_of(path)) {
    std::vector<std::string> w = words(l);
    if (w.size() < 3 || w[0] != "REACTION") continue;
    avgpu_reaction r;
    memset(&r, 0, sizeof(r));
    auto t = task.find(w[2]);
    if (t == task.end()) die("task outside logic-9: " + w[2]);
    r.task = t->second;
    r.type = AVGPU_PROC_ADD;
    r.value = 1.0;
    r.max_number = 1.0;
    r.max_count = INT32_MAX;
    r.max_fraction = 1.0;
    r.depletable = 1;
    for (size_t k = 3; k < w.size(); k++) {
      std::string spec = w[k];
      const bool req = spec.rfind("requisite:", 0) == 0;
      if (req) r.has_requisite = 1;
      std::stringstream parts(spec.substr(spec.find(':') + 1));
      std::string kv;
      while (std::getline(parts, kv, ':')) {
        const size_t eq = kv.find('=');
        if (eq == std::string::npos) continue;
        const std::string key = kv.substr(0, eq), val = kv.substr(eq + 1);
        if (!req && key == "value") r.value = atof(val.c_str());
        else if (!req && key == "type") r.type = val == "pow" ? AVGPU_PROC_POW : (val == "mult" ? AVGPU_PROC_MULT : AVGPU_PROC_ADD);
        else if (!req && key == "max") r.max_number = atof(val.c_str());
        else if (!req && key == "min") r.min_number = atof(val.c_str());
        else if (!req && key == "frac") r.max_fraction = atof(val.c_str());
        else if (!req && key == "resource") die("resource processes need avgpu_load_resources (use the Python driver)");
        else if (req && key == "max_count") r.max_count = atoi(val.c_str());
        else if (req && key == "min_count") r.min_count = atoi(val.c_str());
      }
    }
    out.push_back(r);
  }
  return out;
}

// ---- population: genotype rows of a .pop file (cPopulation::LoadPopulation's
// input, main/cPopulation.cc:6723-7000); genome letters index the instset
struct Genotype {
  std::vector<uint8_t> genome;
  double merit;
  int count;
};

std::vector<Genotype> read_pop(const std::string& path) {
  std::vector<std::string> cols;
  std::vector<Genotype> out;
  for (const std::string& l : lines_of(path)) {
    if (l.rfind("#format", 0) == 0) {
      cols = words(l.substr(1));
      cols.erase(cols.begin());
      continue;
    }
    std::vector<std::string> w = words(l);
    if (w.empty() || cols.empty()) continue;
    Genotype g{{}, 0.0, 0};
    for (size_t k = 0; k < cols.size() && k < w.size(); k++) {
      if (cols[k] == "num_cpus" || cols[k] == "num_units") g.count = atoi(w[k].c_str());
      else if (cols[k] == "merit") g.merit = atof(w[k].c_str());
      else if (cols[k] == "sequence")
        for (char ch : w[k]) g.genome.push_back((uint8_t)(ch >= 'a' ? ch - 'a' : 26 + ch - 'A'));
    }
    out.push_back(g);
  }
  return out;
}

// ---- one strip and the exchanges ------------------------------------------
struct Tile {
  avgpu_world* h = nullptr;
  int64_t n_part = 0, halo_bytes = 0, rec_bytes = 0, res_bytes = 0;
  double* part = nullptr;
  double* gathered = nullptr;
  uint8_t* halo_send[2] = {}; uint8_t* halo_recv[2] = {};
  uint8_t* rec_send[2] = {};  uint8_t* rec_recv[2] = {};
  double* res_send[2] = {};   double* res_recv[2] = {};
  uint64_t* cons = nullptr;
};

enum class Kind { Halo, Records, Resources };

struct Transport {
  virtual ~Transport() = default;
  virtual void all_gather(std::vector<Tile>& t, hipStream_t s) = 0;
  virtual void exchange(std::vector<Tile>& t, Kind k, hipStream_t s) = 0;
  // an exchange the stream's next kernels run beside: issued by
  // exchange_begin, joined into s by exchange_end
  virtual void exchange_begin(std::vector<Tile>& t, Kind k, hipStream_t s) { exchange(t, k, s); }
  virtual void exchange_end(hipStream_t s) {}
  virtual void all_reduce_sum(std::vector<Tile>& t, hipStream_t s) = 0;
};

void buffers(Tile& t, Kind k, void** send, void** recv, size_t& bytes) {
  if (k == Kind::Halo) { send[0] = t.halo_send[0]; send[1] = t.halo_send[1]; recv[0] = t.halo_recv[0]; recv[1] = t.halo_recv[1]; bytes = t.halo_bytes; }
  if (k == Kind::Records) { send[0] = t.rec_send[0]; send[1] = t.rec_send[1]; recv[0] = t.rec_recv[0]; recv[1] = t.rec_recv[1]; bytes = t.rec_bytes; }
  if (k == Kind::Resources) { send[0] = t.res_send[0]; send[1] = t.res_send[1]; recv[0] = t.res_recv[0]; recv[1] = t.res_recv[1]; bytes = t.res_bytes; }
}

// all strips in this process: device copies in tile order on the one stream
struct Loopback : Transport {
  void all_gather(std::vector<Tile>& t, hipStream_t s) override {
    for (size_t i = 0; i < t.size(); i++)
      for (size_t j = 0; j < t.size(); j++)
        HIP_OK(hipMemcpyAsync(t[i].gathered + j * t[j].n_part, t[j].part, t[j].n_part * 8,
                              hipMemcpyDeviceToDevice, s));
  }
  void exchange(std::vector<Tile>& t, Kind k, hipStream_t s) override {
    const size_t T = t.size();
    for (size_t i = 0; i < T; i++) {
      Tile &up = t[(i + T - 1) % T], &down = t[(i + 1) % T];
      void *us[2], *ur[2], *ds[2], *dr[2], *ms[2], *mr[2];
      size_t b = 0;
      buffers(up, k, us, ur, b);
      buffers(down, k, ds, dr, b);
      buffers(t[i], k, ms, mr, b);
      if (!b) continue;
      HIP_OK(hipMemcpyAsync(mr[0], us[1], b, hipMemcpyDeviceToDevice, s));   // from the tile above
      HIP_OK(hipMemcpyAsync(mr[1], ds[0], b, hipMemcpyDeviceToDevice, s));   // from the tile below
    }
  }
  void all_reduce_sum(std::vector<Tile>& t, hipStream_t s) override {
    std::vector<uint64_t> tot(AVGPU_MAX_RESOURCES, 0), v(AVGPU_MAX_RESOURCES);
    for (Tile& x : t) {
      HIP_OK(hipMemcpyAsync(v.data(), x.cons, v.size() * 8, hipMemcpyDeviceToHost, s));
      HIP_OK(hipStreamSynchronize(s));
      for (size_t k = 0; k < v.size(); k++) tot[k] += v[k];
    }
    for (Tile& x : t) HIP_OK(hipMemcpyAsync(x.cons, tot.data(), tot.size() * 8, hipMemcpyHostToDevice, s));
  }
};

// one strip per rank: RCCL over xGMI, every call on the world's stream
struct Rccl : Transport {
  ncclComm_t comm;
  int rank, world;
  hipStream_t side = nullptr;           // the overlapped exchange's stream
  hipEvent_t issued = nullptr, done = nullptr;
  Rccl(ncclComm_t c, int r, int w) : comm(c), rank(r), world(w) {
    HIP_OK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&issued, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  }
  ~Rccl() override {
    (void)hipEventDestroy(issued);
    (void)hipEventDestroy(done);
    (void)hipStreamDestroy(side);
  }
  void exchange_begin(std::vector<Tile>& t, Kind k, hipStream_t s) override {
    HIP_OK(hipEventRecord(issued, s));
    HIP_OK(hipStreamWaitEvent(side, issued, 0));
    exchange(t, k, side);
    HIP_OK(hipEventRecord(done, side));
  }
  void exchange_end(hipStream_t s) override { HIP_OK(hipStreamWaitEvent(s, done, 0)); }
  void all_gather(std::vector<Tile>& t, hipStream_t s) override {
    NCCL_OK(ncclAllGather(t[0].part, t[0].gathered, t[0].n_part, ncclFloat64, comm, s));
  }
  void exchange(std::vector<Tile>& t, Kind k, hipStream_t s) override {
    void *send[2], *recv[2];
    size_t b = 0;
    buffers(t[0], k, send, recv, b);
    if (!b) return;
    const int up = (rank + world - 1) % world, down = (rank + 1) % world;
    // sends [to above, to below], receives [from below, from above]: with two
    // strips both peers are one rank, and a pair's messages match in issue order
    NCCL_OK(ncclGroupStart());
    NCCL_OK(ncclSend(send[0], b, ncclUint8, up, comm, s));
    NCCL_OK(ncclSend(send[1], b, ncclUint8, down, comm, s));
    NCCL_OK(ncclRecv(recv[1], b, ncclUint8, down, comm, s));
    NCCL_OK(ncclRecv(recv[0], b, ncclUint8, up, comm, s));
    NCCL_OK(ncclGroupEnd());
  }
  void all_reduce_sum(std::vector<Tile>& t, hipStream_t s) override {
    NCCL_OK(ncclAllReduce(t[0].cons, t[0].cons, AVGPU_MAX_RESOURCES, ncclUint64, ncclSum, comm, s));
  }
};

template <typename T>
T* dalloc(size_t count) {
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(count * sizeof(T), 16)));
  HIP_OK(hipMemset(p, 0, std::max<size_t>(count * sizeof(T), 16)));
  return (T*)p;
}

void attach(Tile& t, int ntiles) {
  int64_t pb = 0, hb = 0, rb = 0, sb = 0;
  AV_OK(avgpu_tile_buffer_bytes(t.h, &pb, &hb, &rb));
  t.n_part = pb / 8;
  t.halo_bytes = hb;
  t.rec_bytes = rb;
  t.part = dalloc<double>(t.n_part);
  t.gathered = dalloc<double>(t.n_part * ntiles);
  for (int d = 0; d < 2; d++) {
    t.halo_send[d] = dalloc<uint8_t>(hb); t.halo_recv[d] = dalloc<uint8_t>(hb);
    t.rec_send[d] = dalloc<uint8_t>(rb);  t.rec_recv[d] = dalloc<uint8_t>(rb);
  }
  AV_OK(avgpu_set_tile_buffers(t.h, t.halo_send[0], t.halo_send[1], t.halo_recv[0], t.halo_recv[1],
                               t.rec_send[0], t.rec_send[1], t.rec_recv[0], t.rec_recv[1]));
  AV_OK(avgpu_tile_res_bytes(t.h, &sb));
  t.res_bytes = sb;
  for (int d = 0; d < 2; d++) {
    t.res_send[d] = dalloc<double>(std::max<int64_t>(1, sb / 8));
    t.res_recv[d] = dalloc<double>(std::max<int64_t>(1, sb / 8));
  }
  AV_OK(avgpu_set_tile_res_buffers(t.h, t.res_send[0], t.res_send[1], t.res_recv[0], t.res_recv[1]));
  t.cons = dalloc<uint64_t>(AVGPU_MAX_RESOURCES);
}

// the per-update schedule of include/avida_gpu.h ("strip tiles"): the
// update's batch steps K from the gathered predictors (avgpu_tile_steps, the
// same on every strip), then per step the placement protocol
void update(std::vector<Tile>& tiles, Transport& tr, hipStream_t s) {
  int ntiles_total = (int)tiles.size();
  if (auto* r = dynamic_cast<Rccl*>(&tr)) ntiles_total = r->world;
  for (Tile& t : tiles) AV_OK(avgpu_tile_partials(t.h, t.part));
  tr.all_gather(tiles, s);
  int K = 1;
  AV_OK(avgpu_tile_steps(tiles[0].h, tiles[0].gathered, ntiles_total, &K));
  for (int sub = 0; sub < K; sub++) {
    if (sub > 0) {
      for (Tile& t : tiles) AV_OK(avgpu_tile_partials(t.h, t.part));
      tr.all_gather(tiles, s);
    }
    if (sub == 0 && tiles[0].res_bytes > 0) tr.exchange(tiles, Kind::Resources, s);
    for (Tile& t : tiles) AV_OK(avgpu_tile_begin_step(t.h, t.gathered, ntiles_total, sub, K));
    tr.exchange(tiles, Kind::Halo, s);
    // round 0's picks and kill times, then the cancellations and round 0's
    // claims (phase 3, with the neighbours' kill times on the edge rows); then
    // one launch and one exchange per placement round (both strips resolve each
    // edge cell alike, at the start of the next round's launch)
    const int steps[5][2] = {{0, 0}, {0, 3}, {1, 0}, {2, 0}, {3, 0}};
    for (const auto& st : steps) {
      for (Tile& t : tiles) AV_OK(avgpu_tile_place(t.h, st[0], st[1]));
      tr.exchange(tiles, Kind::Halo, s);
    }
    for (Tile& t : tiles) AV_OK(avgpu_tile_place(t.h, 3, 1));   // last resolve, records packed
    tr.exchange_begin(tiles, Kind::Records, s);
    for (Tile& t : tiles) AV_OK(avgpu_tile_place(t.h, 3, 2));   // own winners, beside the exchange
    tr.exchange_end(s);
    for (Tile& t : tiles) AV_OK(avgpu_tile_finish(t.h, nullptr));   // remote offspring, newborn pass
    int pools = 0;
    for (Tile& t : tiles) pools = avgpu_tile_res_cons(t.h, t.cons);
    if (pools > 0) {
      tr.all_reduce_sum(tiles, s);
      for (Tile& t : tiles) AV_OK(avgpu_tile_res_settle(t.h, t.cons));
    }
  }
}

struct Args {
  std::string config = ".";
  int side = 1024, strips = 1, updates = 50, burn_in = 150, gpus = 1;
  int sub_updates = 0;       // avgpu_cfg.sub_updates (0: adaptive batch steps)
  uint64_t seed = 101;
  bool untiled = false;
  bool rccl = false;         // RCCL even for one rank
  bool independent = false;  // one whole world per rank, scheduler totals all-reduced
};

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; i++) {
    std::string k = argv[i];
    auto val = [&]() -> std::string { if (i + 1 >= argc) die("missing value for " + k); return argv[++i]; };
    if (k == "--config") a.config = val();
    else if (k == "--side") a.side = atoi(val().c_str());
    else if (k == "--strips") a.strips = atoi(val().c_str());
    else if (k == "--updates") a.updates = atoi(val().c_str());
    else if (k == "--burn-in") a.burn_in = atoi(val().c_str());
    else if (k == "--seed") a.seed = strtoull(val().c_str(), nullptr, 10);
    else if (k == "--gpus") a.gpus = atoi(val().c_str());
    else if (k == "--sub-updates") a.sub_updates = atoi(val().c_str());
    else if (k == "--untiled") a.untiled = true;
    else if (k == "--rccl") a.rccl = true;
    else if (k == "--independent") a.independent = true;
    else if (k == "--help" || k == "-h") {
      printf("usage: avgpu_strips --config DIR [--side N] [--strips T] [--updates U] [--burn-in B]\n"
             "                    [--seed S] [--gpus N] [--untiled] [--rccl] [--independent]\n"
             "                    [--sub-updates K]\n");
      exit(0);
    } else die("unknown option " + k);
  }
  return a;
}

int env_int(const char* k, int dflt) {
  const char* v = getenv(k);
  return v ? atoi(v) : dflt;
}

// rank 0's RCCL unique id to the other ranks of this node through a file
ncclUniqueId share_id(int rank) {
  ncclUniqueId id;
  const std::string path = std::string("/tmp/avgpu_strips_id_") + (getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "0") +
                           "_" + std::to_string(getppid());
  if (rank == 0) {
    NCCL_OK(ncclGetUniqueId(&id));
    const std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(&id, sizeof(id), 1, f) != 1) die("cannot write " + tmp);
    fclose(f);
    rename(tmp.c_str(), path.c_str());
  } else {
    for (int tries = 0;; tries++) {
      FILE* f = fopen(path.c_str(), "rb");
      if (f && fread(&id, sizeof(id), 1, f) == 1) { fclose(f); break; }
      if (f) fclose(f);
      if (tries > 6000) die("no RCCL id from rank 0 at " + path);
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  return id;
}

// --gpus N: start the N ranks (before this process touches the GPU)
int launch_ranks(int argc, char** argv, int n) {
  std::vector<pid_t> kids;
  for (int r = 0; r < n; r++) {
    const pid_t p = fork();
    if (p < 0) die("fork failed");
    if (p == 0) {
      setenv("RANK", std::to_string(r).c_str(), 1);
      setenv("LOCAL_RANK", std::to_string(r).c_str(), 1);
      setenv("WORLD_SIZE", std::to_string(n).c_str(), 1);
      execv("/proc/self/exe", argv);
      _exit(127);
    }
    kids.push_back(p);
  }
  int rc = 0;
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  (void)argc;
  return rc;
}

uint64_t digest_of(avgpu_world* h, int64_t n, int64_t first_global) {
  std::vector<uint64_t> d(n);
  AV_OK(avgpu_state_digests(h, 0, n, d.data()));
  uint64_t acc = 0;
  for (int64_t i = 0; i < n; i++) acc += d[i] * (2 * (uint64_t)(first_global + i) + 1);
  return acc;
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  if (a.gpus > 1 && !getenv("RANK")) return launch_ranks(argc, argv, a.gpus);
  const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1), local = env_int("LOCAL_RANK", 0);
  const bool multi = world > 1 || a.rccl;
  if (multi && a.strips != 1) die("one strip per rank with more than one rank");
  if (a.independent && !multi) die("--independent needs ranks (--gpus N or --rccl)");
  if (a.independent) a.untiled = true;
  HIP_OK(hipSetDevice(local));
  hipStream_t s;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  InstSet is = read_instset(a.config + "/instset-classic.cfg");
  std::vector<avgpu_reaction> env = read_environment(a.config + "/environment-logic9.cfg");
  std::vector<Genotype> gts = read_pop(a.config + "/detail-50000.pop");
  std::vector<const Genotype*> pool;
  for (const Genotype& g : gts)
    for (int k = 0; k < g.count; k++) pool.push_back(&g);
  if (pool.empty()) die("empty genotype pool");

  const int T = a.independent ? 1 : (multi ? world : a.strips);   // strips of the torus
  const int local_tiles = multi ? 1 : (a.untiled ? 1 : a.strips);
  const int64_t side = a.side, n = side * side * (a.untiled && !a.independent ? a.strips : 1);
  avgpu_cfg cfg;
  avgpu_cfg_defaults(&cfg);
  cfg.world_x = (int32_t)side;
  cfg.world_y = (int32_t)(side * T);
  cfg.seed = a.seed + (a.independent ? (uint64_t)rank : 0);   // independent worlds: a run per seed
  cfg.sub_updates = a.sub_updates;

  std::vector<Tile> tiles(local_tiles);
  for (int k = 0; k < local_tiles; k++) {
    Tile& t = tiles[k];
    t.h = avgpu_create(&cfg, local, n);
    if (!t.h) die(std::string("avgpu_create: ") + avgpu_last_error());
    AV_OK(avgpu_set_stream(t.h, s));
    AV_OK(avgpu_load_instset(t.h, (int)is.handler.size(), is.handler.data(), is.redundancy.data()));
    AV_OK(avgpu_load_env(t.h, (int)env.size(), env.data()));
    const int strip = multi && !a.independent ? rank : k;
    if (!a.untiled) {
      AV_OK(avgpu_set_tile(t.h, (int64_t)strip * side, 0));
      attach(t, T);
    }
    // every cell from the genotype pool (bench.py _genomes_for), keyed by global cell id
    const int64_t first = a.untiled ? 0 : (int64_t)strip * n;
    std::vector<uint8_t> blob;
    std::vector<int32_t> lens(n);
    std::vector<double> merits(n);
    for (int64_t i = 0; i < n; i++) {
      const uint64_t idx = ((uint64_t)(i + first) * 2654435761ull) % (uint64_t)pool.size();
      const Genotype* g = pool[idx];
      blob.insert(blob.end(), g->genome.begin(), g->genome.end());
      lens[i] = (int32_t)g->genome.size();
      merits[i] = g->merit;
    }
    AV_OK(avgpu_set_orgs(t.h, 0, n, blob.data(), lens.data(), merits.data(), nullptr, 0));
  }

  ncclComm_t comm = nullptr;
  std::unique_ptr<Transport> tr;
  if (multi) {
    ncclUniqueId id = share_id(rank);
    NCCL_OK(ncclCommInitRank(&comm, world, id, rank));
    tr.reset(new Rccl(comm, rank, world));
  } else {
    tr.reset(new Loopback());
  }
  double* dtot = dalloc<double>(2);
  auto step = [&]() {
    if (a.independent) {
      AV_OK(avgpu_update_totals(tiles[0].h, dtot));
      NCCL_OK(ncclAllReduce(dtot, dtot, 2, ncclFloat64, ncclSum, comm, s));
      AV_OK(avgpu_update_run(tiles[0].h, dtot, nullptr));
    } else if (a.untiled) {
      AV_OK(avgpu_run_update(tiles[0].h, nullptr));
    } else {
      update(tiles, *tr, s);
    }
  };
  for (int u = 0; u < a.burn_in; u++) step();
  HIP_OK(hipStreamSynchronize(s));
  avgpu_update_stats s0, s1;
  int64_t i0 = 0, i1 = 0;
  for (Tile& t : tiles) { AV_OK(avgpu_get_stats(t.h, &s0)); i0 += s0.cum_insts_executed; }
  const auto t0 = std::chrono::steady_clock::now();
  for (int u = 0; u < a.updates; u++) step();
  HIP_OK(hipStreamSynchronize(s));
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int64_t orgs = 0;
  for (Tile& t : tiles) { AV_OK(avgpu_get_stats(t.h, &s1)); i1 += s1.cum_insts_executed; orgs += s1.num_organisms; }
  uint64_t dig = 0;
  for (int k = 0; k < local_tiles; k++) {
    const int strip = multi && !a.independent ? rank : k;
    dig += digest_of(tiles[k].h, n, a.untiled ? 0 : (int64_t)strip * n);
  }
  // totals over ranks (time: the slowest rank)
  double v[4] = {dt, (double)(i1 - i0), (double)orgs, (double)dig};
  if (multi) {
    double* d = dalloc<double>(4);
    HIP_OK(hipMemcpyAsync(d, v, sizeof(v), hipMemcpyHostToDevice, s));
    NCCL_OK(ncclAllReduce(d + 1, d + 1, 2, ncclFloat64, ncclSum, comm, s));
    NCCL_OK(ncclAllReduce(d, d, 1, ncclFloat64, ncclMax, comm, s));
    HIP_OK(hipMemcpyAsync(v, d, 3 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  if (rank == 0)
    printf("{\"tool\": \"avgpu_strips\", \"ranks\": %d, \"strips\": %d, \"untiled\": %s, \"side\": %lld, "
           "\"updates\": %d, \"ms_per_update\": %.4f, \"organism_instructions_per_s\": %.6g, "
           "\"organisms\": %lld, \"digest_rank0\": \"%016llx\"}\n",
           world, T, a.untiled ? "true" : "false", (long long)side, a.updates, 1e3 * v[0] / a.updates,
           v[1] / v[0], (long long)v[2], (unsigned long long)dig);
  for (Tile& t : tiles) avgpu_destroy(t.h);
  if (comm) ncclCommDestroy(comm);
  return 0;
}

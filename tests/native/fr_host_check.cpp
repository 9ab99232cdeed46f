// Test driver for the engine's host C++ (csrc/fr_sampler.cpp, fr_io.cpp, fr_error.cpp,
// fr_comm.cpp) built with -fsanitize=address,undefined (make -C csrc asan).  Test infrastructure:
// tests/test_asan_cpu.py writes inputs as raw little-endian arrays, runs one subcommand, and
// compares what it writes back with the regular library's results on the same inputs.  Every
// input array is read into a heap block of exactly its size, so an out-of-bounds read by the code
// under test is an AddressSanitizer report (the driver then exits non-zero).
//
//   fr_host_check neg  <dir>                       fr_sampler_negatives(_perm)
//   fr_host_check io   <path> <mode> <threads> <outdir>   fr_io_open + fr_io_fill
//   fr_host_check cand <dir> <threads>             fr_io_remove_positives + fr_io_candidates
//   fr_host_check comm                             fr_comm_* argument checks (no device work)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "fr_engine.h"

namespace {

template <class T>
bool read_arr(const std::string& path, std::vector<T>* out) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) return false;
  const std::streamsize n = f.tellg();
  f.seekg(0);
  out->assign(size_t(n) / sizeof(T), T());
  // an empty vector's data() may be null: the exact-size contract holds for non-empty arrays
  return out->empty() || bool(f.read(reinterpret_cast<char*>(out->data()), std::streamsize(out->size() * sizeof(T))));
}

template <class T>
void write_arr(const std::string& path, const T* p, size_t n) {
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(p), std::streamsize(n * sizeof(T)));
}

void write_rc(const std::string& dir, int rc, int64_t extra = 0) {
  std::ofstream f(dir + "/rc.txt");
  f << rc << " " << extra << "\n" << (rc ? fr_last_error() : "") << "\n";
}

// heap copies of exact size (nullptr for an empty array: the callee must not read it)
template <class T>
T* exact(std::vector<T>& v) { return v.empty() ? nullptr : v.data(); }

int cmd_neg(const std::string& dir) {
  std::vector<uint32_t> key;
  std::vector<int32_t> pos;
  std::vector<int64_t> args, users, perm, ep, ei, e2p, e2i;
  if (!read_arr(dir + "/key.u32", &key) || !read_arr(dir + "/pos.i32", &pos) || !read_arr(dir + "/args.i64", &args) ||
      key.size() != 624 || pos.size() != 1 || args.size() != 4)
    return 2;
  read_arr(dir + "/users.i64", &users);
  const bool has_perm = read_arr(dir + "/perm.i64", &perm);
  read_arr(dir + "/excl_ptr.i64", &ep);
  read_arr(dir + "/excl_items.i64", &ei);
  const bool has2 = read_arr(dir + "/excl2_ptr.i64", &e2p);
  read_arr(dir + "/excl2_items.i64", &e2i);
  const int64_t num_items = args[0], n = args[1], n_users = args[2], n_pairs = args[3];
  std::vector<int64_t> out(static_cast<size_t>(n > 0 ? n : 0), -7);
  const int rc = has_perm
      ? fr_sampler_negatives_perm(key.data(), pos.data(), num_items, exact(users), n_pairs, exact(perm), n, n_users,
                                  exact(ep), exact(ei), has2 ? exact(e2p) : nullptr, has2 ? exact(e2i) : nullptr,
                                  exact(out))
      : fr_sampler_negatives(key.data(), pos.data(), num_items, exact(users), n, n_users, exact(ep), exact(ei),
                             has2 ? exact(e2p) : nullptr, has2 ? exact(e2i) : nullptr, exact(out));
  write_rc(dir, rc);
  write_arr(dir + "/out.i64", out.data(), out.size());
  write_arr(dir + "/key_out.u32", key.data(), key.size());
  write_arr(dir + "/pos_out.i32", pos.data(), pos.size());
  return 0;
}

int cmd_io(const std::string& path, int mode, int threads, const std::string& outdir) {
  fr_io_table* t = nullptr;
  int64_t rows = 0, values = 0, bad = 0;
  int rc = fr_io_open(path.c_str(), mode, threads, &t, &rows, &values);
  if (rc != FR_OK) {
    write_rc(outdir, rc);
    return 0;
  }
  std::vector<int64_t> vals(static_cast<size_t>(values)), offs(mode == FR_IO_NEGATIVE ? static_cast<size_t>(rows) + 1 : 0);
  std::vector<double> aux(mode == FR_IO_RATING ? static_cast<size_t>(rows) : 0);
  rc = fr_io_fill(t, exact(vals), exact(offs), exact(aux), &bad);
  fr_io_close(t);
  write_rc(outdir, rc, bad);
  write_arr(outdir + "/values.i64", vals.data(), vals.size());
  write_arr(outdir + "/offsets.i64", offs.data(), offs.size());
  write_arr(outdir + "/aux.f64", aux.data(), aux.size());
  return 0;
}

int cmd_cand(const std::string& dir, int threads) {
  std::vector<int64_t> neg, neg_off, pos, pos_off, users;
  std::vector<uint8_t> alive;
  if (!read_arr(dir + "/neg.i64", &neg) || !read_arr(dir + "/neg_off.i64", &neg_off) ||
      !read_arr(dir + "/pos.i64", &pos) || !read_arr(dir + "/pos_off.i64", &pos_off) ||
      !read_arr(dir + "/users.i64", &users) || neg_off.empty() || pos_off.size() != neg_off.size())
    return 2;
  alive.assign(neg.size(), 1);
  const int64_t n_users = int64_t(neg_off.size()) - 1;
  std::vector<int64_t> lens(static_cast<size_t>(n_users));
  int64_t total = 0;
  int rc = fr_io_remove_positives(exact(neg), neg_off.data(), exact(alive), exact(pos), pos_off.data(), n_users,
                                  exact(lens), &total, threads);
  if (rc == FR_OK) {
    std::vector<int64_t> cand_off(static_cast<size_t>(n_users) + 1, 0);
    for (int64_t u = 0; u < n_users; ++u) cand_off[size_t(u) + 1] = cand_off[size_t(u)] + lens[size_t(u)];
    std::vector<int64_t> ou(static_cast<size_t>(total)), oi(static_cast<size_t>(total));
    rc = fr_io_candidates(exact(neg), neg_off.data(), exact(alive), exact(pos), pos_off.data(), exact(users), n_users,
                          cand_off.data(), exact(ou), exact(oi), threads);
    write_arr(dir + "/out_users.i64", ou.data(), ou.size());
    write_arr(dir + "/out_items.i64", oi.data(), oi.size());
  }
  write_rc(dir, rc, total);
  return 0;
}

// argument checks that return before any device or RCCL work (RCCL itself is loaded, when present,
// by the first call: the one part of this driver that maps a system library)
int cmd_comm() {
  int bad = 0;
  auto expect = [&](bool ok, const char* what) {
    if (!ok) {
      std::fprintf(stderr, "comm: %s\n", what);
      ++bad;
    }
  };
  expect(fr_comm_destroy(nullptr) == FR_OK, "destroy(null)");
  const int avail = fr_comm_available();
  const int not_ok = avail ? FR_EINVAL : FR_ENOTSUP;
  float x = 0.f;
  expect(fr_allreduce_f32(nullptr, &x, 1, nullptr) == not_ok, "allreduce(null comm)");
  expect(fr_allgather_f32(nullptr, &x, &x, 1, nullptr) == not_ok, "allgather(null comm)");
  char id[128] = {0};
  void* comm = nullptr;
  expect(fr_comm_init(2, 2, id, &comm) == not_ok, "init(rank out of range)");
  expect(fr_comm_init(0, 1, nullptr, &comm) == not_ok, "init(null id)");
  expect(fr_comm_unique_id(id, 4) == not_ok, "unique_id(short buffer)");
  expect(fr_comm_unique_id_bytes() == 128, "unique_id_bytes");
  std::printf("comm available=%d failures=%d\n", avail, bad);
  return bad ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string cmd = argv[1];
  if (cmd == "neg" && argc == 3) return cmd_neg(argv[2]);
  if (cmd == "io" && argc == 6) return cmd_io(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argv[5]);
  if (cmd == "cand" && argc == 4) return cmd_cand(argv[2], std::atoi(argv[3]));
  if (cmd == "comm" && argc == 2) return cmd_comm();
  return 2;
}

// GPU text ingest: edge-list files and -v label files
// parsed in HBM.
//
// Reference semantics restated:
//   * edge lines: `std::istringstream(line) >> src >> dst` (parallel_edge_list_reader.hpp:242-266),
//     lines that do not yield two numbers are skipped, -u 1 adds (dst, src) after every (src, dst)
//     (ingest_edge_list.cpp:92,115,164-240); ids above 2^32 - 2 are refused (u32 CSR columns);
//   * label lines: `iss >> vid >> label` on zero-initialised values (vertex_data_db.hpp:176-185):
//     a line that does not parse sets label 0 on vertex 0 (or on the vid it did read), files are
//     applied in name order and a later line wins (vertex_data_db.hpp:197-257);
//   * numbers follow num_get in the "C" locale: white space skipped, optional sign ('-' negates
//     modulo 2^64, as strtoull), decimal digits, overflow -> ULLONG_MAX and failure.
//
// MI355X design: the files are streamed through two pinned staging buffers in
// pieces of <= 256 MiB that end at a newline (a helper thread pages the next
// piece in, split over several copy threads, while the device parses the
// current one); per piece, one thread per
// 32-byte window owns the lines that START in its window (a line start is a
// byte after '\n'), parses them in place and, after an exclusive scan of the
// per-window counts (rocPRIM), writes its edges at its own offset: the key
// array is deterministic and no atomics touch it.  Keys (src << B | dst, B =
// bit width of the largest id) are then radix-sorted on 2B bits and turned
// into the row-sorted CSR with multiplicity by the same pass the R-MAT builder
// uses; symmetry is decided by sorting the swapped keys and comparing them
// with the sorted keys (equal multisets <=> symmetric), and that swapped,
// sorted array is the in-row CSR a directed graph's superstep 0 scans.
// Labels: two passes per piece, atomicMax of the line's global byte ordinal
// per vertex, then the winning line writes its label (last write wins).

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <iostream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "pm_ingest.hpp"
#include "pm_internal.hpp"

namespace pm {

namespace {

constexpr uint64_t kWin = 32;                // bytes of line starts owned by one thread
constexpr uint64_t kPiece = 256ull << 20;    // text bytes per upload (ends after a '\n')
constexpr unsigned kThreads = 256;
constexpr uint64_t kMaxId = 0xFFFFFFFEull;   // u32 columns; 0xFFFFFFFF marks padding on the device

struct Buf {
  void* p = nullptr;
  ~Buf() { reset(); }
  template <typename T>
  T* alloc(uint64_t n) {
    reset();
    PM_HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(n, 1) * sizeof(T)));
    return static_cast<T*>(p);
  }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
  }
  template <typename T>
  T* get() const { return static_cast<T*>(p); }
};

struct PinnedBuf {
  char* p = nullptr;
  explicit PinnedBuf(uint64_t bytes) { PM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p), bytes)); }
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// The files in order, cut into pieces that end with '\n' (a file's last line
// gets one appended, as std::getline reads it without one).  Files are read
// through read-only mappings.
class TextPieces {
 public:
  explicit TextPieces(const std::vector<std::string>& files) : files_(files) {}
  ~TextPieces() { close(); }
  uint64_t total_bytes() const {
    uint64_t t = 0;
    for (const auto& f : files_) {
      struct stat st;
      if (::stat(f.c_str(), &st) == 0) t += static_cast<uint64_t>(st.st_size) + 1;
    }
    return t;
  }
  // copies the next piece into dst (capacity cap >= 2); returns its length, 0 at the end
  uint64_t next(char* dst, uint64_t cap) {
    for (;;) {
      if (!map_) {
        if (fi_ >= files_.size()) return 0;
        if (!open(files_[fi_++])) continue;
      }
      if (pos_ >= len_) {
        close();
        continue;
      }
      const char* s = map_ + pos_;
      uint64_t take = std::min<uint64_t>(len_ - pos_, cap - 1);
      if (pos_ + take < len_) {
        const void* nl = memrchr(s, '\n', take);
        if (!nl) throw std::runtime_error("ingest: a text line is longer than the upload piece");
        take = static_cast<uint64_t>(static_cast<const char*>(nl) - s) + 1;
      }
      par_copy(dst, s, take);
      pos_ += take;
      if (dst[take - 1] != '\n') dst[take++] = '\n';
      return take;
    }
  }

 private:
  // page-in + copy of a piece split over kCopyThreads threads (one thread copies a mapped file at a few GB/s)
  static void par_copy(char* dst, const char* src, uint64_t n) {
    constexpr unsigned kCopyThreads = 8;
    constexpr uint64_t kMinChunk = 8ull << 20;
    const unsigned t = static_cast<unsigned>(std::min<uint64_t>(kCopyThreads, (n + kMinChunk - 1) / kMinChunk));
    if (t <= 1) {
      std::memcpy(dst, src, n);
      return;
    }
    const uint64_t chunk = (n + t - 1) / t;
    std::vector<std::thread> th;
    for (unsigned i = 1; i < t; ++i) {
      const uint64_t b = i * chunk, e = std::min(n, b + chunk);
      if (b < e) th.emplace_back([=] { std::memcpy(dst + b, src + b, e - b); });
    }
    std::memcpy(dst, src, std::min(n, chunk));
    for (auto& x : th) x.join();
  }
  bool open(const std::string& path) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) {
      std::cerr << "Error opening filename: " << path << std::endl;  // the reference goes on
      return false;
    }
    struct stat st;
    if (::fstat(fd, &st) != 0 || st.st_size == 0) {
      ::close(fd);
      return false;
    }
    void* m = ::mmap(nullptr, static_cast<size_t>(st.st_size), PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) throw std::runtime_error("ingest: cannot map " + path);
    (void)::madvise(m, static_cast<size_t>(st.st_size), MADV_SEQUENTIAL);
    map_ = static_cast<const char*>(m);
    len_ = static_cast<uint64_t>(st.st_size);
    pos_ = 0;
    return true;
  }
  void close() {
    if (map_) ::munmap(const_cast<char*>(map_), len_);
    map_ = nullptr;
    len_ = pos_ = 0;
  }
  const std::vector<std::string>& files_;
  size_t fi_ = 0;
  const char* map_ = nullptr;
  uint64_t len_ = 0, pos_ = 0;
};

// Double-buffered staging: pieces alternate between two pinned buffers; the
// next piece is filled on a helper thread while the device works on the
// current one.  A buffer is refilled only after the upload that read it has
// completed (its event).
class PieceFeeder {
 public:
  PieceFeeder(TextPieces& pieces, uint64_t cap) : pieces_(pieces), cap_(cap), a_(cap), b_(cap) {
    for (auto& e : ev_) PM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    fill(0);
  }
  ~PieceFeeder() {
    if (worker_.joinable()) worker_.join();
    for (auto& e : ev_) (void)hipEventDestroy(e);
  }
  // the current piece (its length; 0 at the end) and its pinned bytes
  uint64_t wait() {
    if (worker_.joinable()) worker_.join();
    if (err_) std::rethrow_exception(err_);
    return len_[cur_];
  }
  const char* data() const { return cur_ ? b_.p : a_.p; }
  // enqueues the current piece's upload on s, then starts filling the other buffer with the next piece
  void upload(void* d_dst, hipStream_t s) {
    PM_HIP_CHECK(hipMemcpyAsync(d_dst, data(), len_[cur_], hipMemcpyHostToDevice, s));
    PM_HIP_CHECK(hipEventRecord(ev_[cur_], s));
    cur_ ^= 1;
    fill(cur_);
  }

 private:
  void fill(int i) {
    worker_ = std::thread([this, i] {
      try {
        PM_HIP_CHECK(hipEventSynchronize(ev_[i]));  // the upload that last read buffer i is done
        len_[i] = pieces_.next(i ? b_.p : a_.p, cap_);
      } catch (...) {
        err_ = std::current_exception();
        len_[i] = 0;
      }
    });
  }
  TextPieces& pieces_;
  uint64_t cap_;
  PinnedBuf a_, b_;
  hipEvent_t ev_[2] = {nullptr, nullptr};
  uint64_t len_[2] = {0, 0};
  int cur_ = 0;
  std::thread worker_;
  std::exception_ptr err_;
};

__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// operator>>(unsigned long long&) in the "C" locale, from t[i] up to end.
__device__ __forceinline__ bool get_u64(const uint8_t* __restrict__ t, uint64_t& i, uint64_t end, uint64_t& v) {
  while (i < end && is_space(t[i])) ++i;
  bool neg = false;
  if (i < end && (t[i] == '+' || t[i] == '-')) {
    neg = t[i] == '-';
    ++i;
  }
  uint64_t x = 0;
  bool any = false, ovf = false;
  while (i < end && t[i] >= '0' && t[i] <= '9') {
    const uint64_t d = t[i] - '0';
    if (x > (~0ull - d) / 10) ovf = true;
    else x = x * 10 + d;
    any = true;
    ++i;
  }
  if (!any) {
    v = 0;
    return false;
  }
  if (ovf) {
    v = ~0ull;
    return false;
  }
  v = neg ? 0ull - x : x;
  return true;
}

// Lines [b, e) (e = the '\n') that start in window w of a piece of L bytes whose last byte is '\n'.
template <typename F>
__device__ __forceinline__ void for_lines(const uint8_t* __restrict__ t, uint64_t L, uint64_t w, F&& f) {
  const uint64_t b0 = w * kWin, e0 = min(b0 + kWin, L);
  for (uint64_t i = b0; i < e0; ++i) {
    if (i != 0 && t[i - 1] != '\n') continue;
    uint64_t j = i;
    while (t[j] != '\n') ++j;  // stops at byte L - 1 at the latest
    f(i, j);
    i = j;  // the next line starts at j + 1
  }
}

__device__ __forceinline__ bool edge_of(const uint8_t* __restrict__ t, uint64_t b, uint64_t e, uint64_t& s,
                                        uint64_t& d) {
  uint64_t i = b;
  if (!get_u64(t, i, e, s)) return false;
  return get_u64(t, i, e, d);
}

__global__ __launch_bounds__(kThreads) void k_count_edges(const uint8_t* __restrict__ t, uint64_t L, uint64_t nw,
                                                          uint32_t* __restrict__ cnt) {
  const uint64_t w = blockIdx.x * uint64_t(kThreads) + threadIdx.x;
  if (w >= nw) return;
  uint32_t c = 0;
  for_lines(t, L, w, [&](uint64_t b, uint64_t e) {
    uint64_t s, d;
    if (edge_of(t, b, e, s, d)) ++c;
  });
  cnt[w] = c;
}

// Writes (src, dst) pairs as (src << 32 | dst) at pos[w]; the largest id and
// an out-of-range flag go to stat[0] (max) / stat[1] (flag) / stat[2] (lines).
__global__ __launch_bounds__(kThreads) void k_emit_edges(const uint8_t* __restrict__ t, uint64_t L, uint64_t nw,
                                                         const uint32_t* __restrict__ pos,
                                                         uint64_t* __restrict__ keys,
                                                         unsigned long long* __restrict__ stat) {
  const uint64_t w = blockIdx.x * uint64_t(kThreads) + threadIdx.x;
  uint64_t mx = 0, lines = 0;
  bool bad = false;
  if (w < nw) {
    uint64_t k = pos[w];
    for_lines(t, L, w, [&](uint64_t b, uint64_t e) {
      ++lines;
      uint64_t s, d;
      if (!edge_of(t, b, e, s, d)) return;
      if (s > kMaxId || d > kMaxId) bad = true;
      keys[k++] = (s << 32) | (d & 0xFFFFFFFFull);
      mx = max(mx, max(s, d));
    });
  }
  for (int o = 32; o; o >>= 1) {
    mx = max(mx, static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(mx), o)));
    lines += static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(lines), o));
  }
  if ((threadIdx.x & 63) == 0) {
    if (mx) atomicMax(&stat[0], static_cast<unsigned long long>(mx));
    if (lines) atomicAdd(&stat[2], static_cast<unsigned long long>(lines));
  }
  if (bad) atomicOr(&stat[1], 1ull);
}

// (s << 32 | d) -> (s << B | d), and with `both` also (d << B | s) at m + i.
__global__ void k_pack_keys(const uint64_t* __restrict__ in, uint64_t m, int B, bool both,
                            uint64_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < m; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t k = in[i], s = k >> 32, d = k & 0xFFFFFFFFull;
    out[i] = (s << B) | d;
    if (both) out[m + i] = (d << B) | s;
  }
}

__global__ void k_swap_keys(const uint64_t* __restrict__ in, uint64_t m, int B, uint64_t* __restrict__ out) {
  const uint64_t mask = (1ull << B) - 1;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < m; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t k = in[i];
    out[i] = ((k & mask) << B) | (k >> B);
  }
}

__global__ void k_keys_differ(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t m,
                              unsigned* __restrict__ flag) {
  bool diff = false;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < m; i += uint64_t(gridDim.x) * blockDim.x)
    diff |= a[i] != b[i];
  if (diff) *flag = 1u;
}

// Sorted keys (s << B | d) -> n + 1 row offsets and the columns (as k_csr_from_keys in pm_rmat.hip).
__global__ void k_csr_from_sorted(const uint64_t* __restrict__ keys, uint64_t m, int B, uint64_t n,
                                  uint64_t* __restrict__ off, uint32_t* __restrict__ col) {
  const uint64_t mask = (1ull << B) - 1;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < m; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t k = keys[i], s = k >> B;
    col[i] = static_cast<uint32_t>(k & mask);
    const uint64_t first = i ? (keys[i - 1] >> B) + 1 : 0;
    for (uint64_t w = first; w <= s; ++w) off[w] = i;
    if (i == m - 1)
      for (uint64_t w = s + 1; w <= n; ++w) off[w] = m;
  }
}

__global__ __launch_bounds__(kThreads) void k_label_lines(const uint8_t* __restrict__ t, uint64_t L, uint64_t nw,
                                                          uint64_t ord0, uint64_t n,
                                                          unsigned long long* __restrict__ win,
                                                          uint64_t* __restrict__ labels, int pass) {
  const uint64_t w = blockIdx.x * uint64_t(kThreads) + threadIdx.x;
  if (w >= nw) return;
  for_lines(t, L, w, [&](uint64_t b, uint64_t e) {
    uint64_t i = b, v = 0, d = 0;
    if (get_u64(t, i, e, v)) (void)get_u64(t, i, e, d);  // a failed label read leaves 0 / ULLONG_MAX
    if (v >= n) return;
    const unsigned long long ord = ord0 + b + 1;
    if (pass == 0) atomicMax(&win[v], ord);
    else if (win[v] == ord) labels[v] = d;
  });
}

// PM_INGEST_PIECE (bytes, >= 64): smaller upload pieces, so that tests cross piece boundaries
uint64_t piece_bytes() {
  if (const char* e = std::getenv("PM_INGEST_PIECE")) return std::max<uint64_t>(64, std::strtoull(e, nullptr, 10));
  return kPiece;
}

unsigned grid_for(uint64_t items, unsigned per, unsigned cap) {
  const uint64_t g = (items + per - 1) / per;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(g, cap)));
}

int bit_width(uint64_t x) {
  int b = 0;
  while (x) {
    ++b;
    x >>= 1;
  }
  return b;
}

// Sorts keys[0..m) on bits [0, bits) in place (alt: scratch of m keys); returns the sorted buffer.
uint64_t* sort_keys(uint64_t* keys, uint64_t* alt, uint64_t m, int bits, hipStream_t s) {
  if (m < 2) return keys;
  rocprim::double_buffer<uint64_t> db(keys, alt);
  size_t tb = 0;
  PM_HIP_CHECK(rocprim::radix_sort_keys(nullptr, tb, db, m, 0u, static_cast<unsigned>(bits), s));
  Buf tmp;
  void* d_tmp = tmp.alloc<char>(tb);
  PM_HIP_CHECK(rocprim::radix_sort_keys(d_tmp, tb, db, m, 0u, static_cast<unsigned>(bits), s));
  PM_HIP_CHECK(hipStreamSynchronize(s));
  return db.current();
}

DevCsr csr_from_sorted(const uint64_t* keys, uint64_t m, int B, uint64_t n, hipStream_t s) {
  DevCsr g;
  g.n = n;
  g.nnz = m;
  PM_HIP_CHECK(hipMalloc(&g.d_off, (n + 1) * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMalloc(&g.d_col, std::max<uint64_t>(m, 1) * sizeof(uint32_t)));
  if (m) {
    hipLaunchKernelGGL(k_csr_from_sorted, dim3(grid_for(m, 256, 1u << 20)), dim3(256), 0, s, keys, m, B, n, g.d_off,
                       g.d_col);
    PM_HIP_CHECK(hipGetLastError());
  } else {
    PM_HIP_CHECK(hipMemsetAsync(g.d_off, 0, (n + 1) * sizeof(uint64_t), s));
  }
  PM_HIP_CHECK(hipStreamSynchronize(s));
  return g;
}

}  // namespace

IngestCsr ingest_edges_device(const std::vector<std::string>& files, bool undirected, bool want_rev,
                              hipStream_t stream) {
  IngestCsr out;
  TextPieces pieces(files);
  const uint64_t total = pieces.total_bytes();
  const uint64_t piece = piece_bytes();
  PinnedBuf tail(64);
  Buf text, cnt, pos, scan_tmp, stat, kf;
  uint8_t* d_text = text.alloc<uint8_t>(piece);
  const uint64_t nw_max = (piece + kWin - 1) / kWin;
  uint32_t* d_cnt = cnt.alloc<uint32_t>(nw_max);
  uint32_t* d_pos = pos.alloc<uint32_t>(nw_max);
  auto* d_stat = stat.alloc<unsigned long long>(4);
  PM_HIP_CHECK(hipMemsetAsync(d_stat, 0, 4 * sizeof(unsigned long long), stream));
  size_t scan_bytes = 0;
  PM_HIP_CHECK(rocprim::exclusive_scan(nullptr, scan_bytes, d_cnt, d_pos, 0u, nw_max, rocprim::plus<uint32_t>(),
                                       stream));
  void* d_scan = scan_tmp.alloc<char>(scan_bytes);
  // forward keys (src << 32 | dst), grown on demand (a line of an edge takes >= 4 bytes)
  uint64_t cap = std::max<uint64_t>(total / 12, 1 << 16), used = 0;
  uint64_t* d_kf = kf.alloc<uint64_t>(cap);
  uint32_t* h_tail = reinterpret_cast<uint32_t*>(tail.p);
  PieceFeeder feed(pieces, piece);
  for (;;) {
    const uint64_t L = feed.wait();
    if (!L) break;
    out.bytes += L;
    // (the previous piece's kernels have completed: the stream was synchronised after them)
    feed.upload(d_text, stream);
    const uint64_t nw = (L + kWin - 1) / kWin;
    hipLaunchKernelGGL(k_count_edges, dim3(grid_for(nw, kThreads, 1u << 30)), dim3(kThreads), 0, stream, d_text, L,
                       nw, d_cnt);
    PM_HIP_CHECK(hipGetLastError());
    PM_HIP_CHECK(rocprim::exclusive_scan(d_scan, scan_bytes, d_cnt, d_pos, 0u, nw, rocprim::plus<uint32_t>(),
                                         stream));
    PM_HIP_CHECK(hipMemcpyAsync(h_tail, d_pos + nw - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    PM_HIP_CHECK(hipMemcpyAsync(h_tail + 1, d_cnt + nw - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    PM_HIP_CHECK(hipStreamSynchronize(stream));
    const uint64_t c = uint64_t(h_tail[0]) + h_tail[1];
    if (used + c > cap) {
      const uint64_t ncap = std::max(2 * cap, used + c);
      Buf grown;
      uint64_t* g = grown.alloc<uint64_t>(ncap);
      PM_HIP_CHECK(hipMemcpyAsync(g, d_kf, used * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
      PM_HIP_CHECK(hipStreamSynchronize(stream));
      std::swap(kf.p, grown.p);
      d_kf = g;
      cap = ncap;
    }
    hipLaunchKernelGGL(k_emit_edges, dim3(grid_for(nw, kThreads, 1u << 30)), dim3(kThreads), 0, stream, d_text, L,
                       nw, d_pos, d_kf + used, d_stat);
    PM_HIP_CHECK(hipGetLastError());
    used += c;
    PM_HIP_CHECK(hipStreamSynchronize(stream));  // d_text is overwritten by the next upload
  }
  unsigned long long hs[4];
  PM_HIP_CHECK(hipMemcpy(hs, d_stat, sizeof(hs), hipMemcpyDeviceToHost));
  if (hs[1]) throw std::runtime_error("vertex id exceeds 32 bits");
  out.lines = hs[2];
  text.reset();
  cnt.reset();
  pos.reset();
  scan_tmp.reset();
  const uint64_t n = used ? hs[0] + 1 : 0;
  const int B = std::max(1, bit_width(n ? n - 1 : 0));
  const uint64_t m = used * (undirected ? 2 : 1);
  Buf ka, kb;
  uint64_t* a = ka.alloc<uint64_t>(m);
  if (used) {
    hipLaunchKernelGGL(k_pack_keys, dim3(grid_for(used, 256, 1u << 20)), dim3(256), 0, stream, d_kf, used, B,
                       undirected, a);
    PM_HIP_CHECK(hipGetLastError());
    PM_HIP_CHECK(hipStreamSynchronize(stream));
  }
  kf.reset();
  uint64_t* b = kb.alloc<uint64_t>(m);
  uint64_t* sorted = sort_keys(a, b, m, 2 * B, stream);
  uint64_t* other = sorted == a ? b : a;
  out.symmetric = true;
  if (!undirected && m) {
    // swapped keys, sorted: equal to the sorted keys <=> every (u,v) has a (v,u) of equal multiplicity
    hipLaunchKernelGGL(k_swap_keys, dim3(grid_for(m, 256, 1u << 20)), dim3(256), 0, stream, sorted, m, B, other);
    PM_HIP_CHECK(hipGetLastError());
    Buf kc;
    uint64_t* c3 = kc.alloc<uint64_t>(m);
    uint64_t* rsorted = sort_keys(other, c3, m, 2 * B, stream);
    unsigned* d_flag = reinterpret_cast<unsigned*>(c3 == rsorted ? other : c3);  // the free scratch
    PM_HIP_CHECK(hipMemsetAsync(d_flag, 0, sizeof(unsigned), stream));
    hipLaunchKernelGGL(k_keys_differ, dim3(grid_for(m, 256, 16384)), dim3(256), 0, stream, sorted, rsorted, m,
                       d_flag);
    PM_HIP_CHECK(hipGetLastError());
    unsigned diff = 0;
    PM_HIP_CHECK(hipMemcpyAsync(&diff, d_flag, sizeof(unsigned), hipMemcpyDeviceToHost, stream));
    PM_HIP_CHECK(hipStreamSynchronize(stream));
    out.symmetric = diff == 0;
    if (!out.symmetric && want_rev) out.rev = csr_from_sorted(rsorted, m, B, n, stream);
  }
  out.fwd = csr_from_sorted(sorted, m, B, n, stream);
  return out;
}

void labels_from_files_device(const std::vector<std::string>& files, uint64_t n, uint64_t* d_labels,
                              hipStream_t stream) {
  TextPieces pieces(files);
  const uint64_t piece = piece_bytes();
  Buf text, win;
  uint8_t* d_text = text.alloc<uint8_t>(piece);
  auto* d_win = win.alloc<unsigned long long>(n);
  PM_HIP_CHECK(hipMemsetAsync(d_win, 0, std::max<uint64_t>(n, 1) * sizeof(unsigned long long), stream));
  PM_HIP_CHECK(hipMemsetAsync(d_labels, 0, std::max<uint64_t>(n, 1) * sizeof(uint64_t), stream));
  uint64_t ord0 = 0;
  PieceFeeder feed(pieces, piece);
  for (;;) {
    const uint64_t L = feed.wait();
    if (!L) break;
    feed.upload(d_text, stream);
    const uint64_t nw = (L + kWin - 1) / kWin;
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(k_label_lines, dim3(grid_for(nw, kThreads, 1u << 30)), dim3(kThreads), 0, stream, d_text,
                         L, nw, ord0, n, d_win, d_labels, pass);
      PM_HIP_CHECK(hipGetLastError());
    }
    ord0 += L;
    PM_HIP_CHECK(hipStreamSynchronize(stream));  // d_text is overwritten by the next upload
  }
}

}  // namespace pm

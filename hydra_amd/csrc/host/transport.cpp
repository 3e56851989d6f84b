// transport.cpp -- minimal TCP transport + rendezvous stores for the host runtime.
//
// One connected socket per pair (full mesh).  Each pair owns a writer thread (FIFO of posted
// sends: header {slot, nbytes} + payload via one sendmsg) and a reader thread (reads a header, waits
// for the FIFO-next posted receive on that pair, then reads the payload straight into it).
// Matching is FIFO per pair; slots are checked (a mismatch is a protocol error).

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <sstream>
#include <thread>

#include "../../../include/hydra/allreduce.h"

namespace hydra {

// ---- stores -------------------------------------------------------------------------------
void HashStore::set(const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> g(mu_);
  kv_[key] = value;
}

std::string HashStore::get(const std::string& key, std::chrono::milliseconds timeout) {
  const auto deadline = std::chrono::steady_clock::now() + timeout;
  for (;;) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = kv_.find(key);
      if (it != kv_.end()) return it->second;
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw IoException("Timed out waiting for store key " + key);
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

void FileStore::set(const std::string& key, const std::string& value) {
  const std::string tmp = dir_ + "/." + key + ".tmp", dst = dir_ + "/" + key;
  {
    std::ofstream f(tmp, std::ios::binary);
    f << value;
  }
  if (::rename(tmp.c_str(), dst.c_str()) != 0)
    throw IoException("FileStore rename failed: " + std::string(std::strerror(errno)));
}

std::string FileStore::get(const std::string& key, std::chrono::milliseconds timeout) {
  const auto deadline = std::chrono::steady_clock::now() + timeout;
  const std::string path = dir_ + "/" + key;
  for (;;) {
    std::ifstream f(path, std::ios::binary);
    if (f) {
      std::stringstream ss;
      ss << f.rdbuf();
      return ss.str();
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw IoException("Timed out waiting for store key " + key);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
}

// ---- pair -----------------------------------------------------------------------------------
struct UnboundBuffer::Op {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::string error;
  char* ptr = nullptr;
  size_t nbytes = 0;
  uint64_t slot = 0;
  void finish(const std::string& err = "") {
    std::lock_guard<std::mutex> g(mu);
    done = true;
    error = err;
    cv.notify_all();
  }
};

namespace transport {

struct Header {
  uint64_t slot;
  uint64_t nbytes;
};

class Pair {
 public:
  Pair(int fd, int self, int peer) : fd_(fd), self_(self), peer_(peer) {
    int one = 1;
    ::setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int buf = 4 << 20;
    ::setsockopt(fd_, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
    ::setsockopt(fd_, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
    writer_ = std::thread([this] { writeLoop(); });
    reader_ = std::thread([this] { readLoop(); });
  }
  ~Pair() { close(); }

  void postSend(std::shared_ptr<UnboundBuffer::Op> op) {
    std::lock_guard<std::mutex> g(mu_);
    if (!error_.empty()) {
      op->finish(error_);
      return;
    }
    sendq_.push_back(std::move(op));
    cv_.notify_all();
  }
  void postRecv(std::shared_ptr<UnboundBuffer::Op> op) {
    std::lock_guard<std::mutex> g(mu_);
    if (!error_.empty()) {
      op->finish(error_);
      return;
    }
    recvq_.push_back(std::move(op));
    cv_.notify_all();
  }
  void close() { abort("Connection closed"); }
  // Fail every pending operation with `e`, refuse new ones, shut the socket and join both
  // threads: when this returns no transport thread touches any operation's memory again -- for
  // EVERY caller: a second, concurrent abort (two timed-out waits, a timeout racing
  // closeConnections) waits until the first one has joined both threads.
  void abort(const std::string& e) {
    fail(e);
    {
      std::unique_lock<std::mutex> l(mu_);
      if (closed_) {
        cv_.wait(l, [&] { return joined_; });
        return;
      }
      closed_ = true;
      cv_.notify_all();
    }
    ::shutdown(fd_, SHUT_RDWR);
    if (writer_.joinable()) writer_.join();
    if (reader_.joinable()) reader_.join();
    ::close(fd_);
    std::lock_guard<std::mutex> g(mu_);
    joined_ = true;
    cv_.notify_all();
  }

 private:
  void fail(const std::string& e) {
    std::deque<std::shared_ptr<UnboundBuffer::Op>> s, r;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (error_.empty()) error_ = e;
      s.swap(sendq_);
      r.swap(recvq_);
      cv_.notify_all();
    }
    for (auto& o : s) o->finish(e);
    for (auto& o : r) o->finish(e);
  }

  // sendmsg with MSG_NOSIGNAL, not writev: a peer that died makes the write fail with EPIPE
  // (-> "Connection closed by peer", IoException at the caller) instead of raising SIGPIPE,
  // which would kill this whole process (the reference's tests ignore SIGPIPE process-wide for
  // the same reason, gloo/gloo/test/main.cc:11-15; the library does not rely on its caller).
  bool writeAll(struct iovec* iov, int n) {
    while (n > 0) {
      struct msghdr m {};
      m.msg_iov = iov;
      m.msg_iovlen = (size_t)n;
      ssize_t w = ::sendmsg(fd_, &m, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      while (n > 0 && (size_t)w >= iov->iov_len) {
        w -= iov->iov_len;
        iov++;
        n--;
      }
      if (n > 0) {
        iov->iov_base = static_cast<char*>(iov->iov_base) + w;
        iov->iov_len -= w;
      }
    }
    return true;
  }

  bool readAll(char* p, size_t len) {
    while (len > 0) {
      ssize_t r = ::recv(fd_, p, len, 0);
      if (r == 0) return false;
      if (r < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      p += r;
      len -= r;
    }
    return true;
  }

  void writeLoop() {
    for (;;) {
      std::shared_ptr<UnboundBuffer::Op> op;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return closed_ || !sendq_.empty(); });
        if (closed_) return;  // abort() already failed whatever was queued
        op = sendq_.front();
        sendq_.pop_front();
      }
      Header h{op->slot, op->nbytes};
      struct iovec iov[2] = {{&h, sizeof(h)}, {op->ptr, op->nbytes}};
      if (!writeAll(iov, op->nbytes ? 2 : 1)) {
        op->finish("Connection closed by peer " + std::to_string(peer_));
        fail("Connection closed by peer " + std::to_string(peer_));
        return;
      }
      op->finish();
    }
  }

  void readLoop() {
    for (;;) {
      Header h;
      if (!readAll(reinterpret_cast<char*>(&h), sizeof(h))) {
        fail("Connection closed by peer " + std::to_string(peer_));
        return;
      }
      std::shared_ptr<UnboundBuffer::Op> op;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return closed_ || !recvq_.empty(); });
        if (closed_) return;
        op = recvq_.front();
        recvq_.pop_front();
      }
      if (op->slot != h.slot || op->nbytes != h.nbytes) {
        std::string e = "protocol error: expected slot " + std::to_string(op->slot) + " bytes " +
                        std::to_string(op->nbytes) + ", got slot " + std::to_string(h.slot) +
                        " bytes " + std::to_string(h.nbytes);
        op->finish(e);
        fail(e);
        return;
      }
      if (!readAll(op->ptr, op->nbytes)) {
        op->finish("Connection closed by peer " + std::to_string(peer_));
        fail("Connection closed by peer " + std::to_string(peer_));
        return;
      }
      op->finish();
    }
  }

  int fd_, self_, peer_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<UnboundBuffer::Op>> sendq_, recvq_;
  bool closed_ = false;
  bool joined_ = false;  // both threads joined and the socket closed (abort() finished)
  std::string error_;
  std::thread writer_, reader_;
};

}  // namespace transport

// ---- context --------------------------------------------------------------------------------
Context::Context(int rank, int size) : rank(rank), size(size) {
  if (size < 1 || rank < 0 || rank >= size) throw EnforceNotMet("invalid rank/size");
  pairs_.resize(size);
}

Context::~Context() {
  closeConnections();
  releaseScratch();
}

void Context::releaseScratch() {
  if (!scratch_) return;
  if (scratch_alloc_.release && !scratch_heap_) scratch_alloc_.release(scratch_);
  else std::free(scratch_);
  scratch_ = nullptr;
  scratch_bytes_ = 0;
}

void Context::setScratchAllocator(ScratchAllocator a) {
  if ((a.alloc == nullptr) != (a.release == nullptr))
    throw EnforceNotMet("scratch allocator needs both alloc and release");
  releaseScratch();
  scratch_alloc_ = a;
}

char* Context::scratch(size_t bytes) {
  if (bytes > scratch_bytes_ || !scratch_) {
    releaseScratch();
    const size_t b = bytes ? bytes : 1;
    scratch_ = scratch_alloc_.alloc ? scratch_alloc_.alloc(b) : nullptr;
    scratch_heap_ = scratch_ == nullptr;  // no allocator, or it declined (e.g. no GPU)
    if (!scratch_) scratch_ = std::malloc(b);
    if (!scratch_) throw EnforceNotMet("scratch allocation of " + std::to_string(b) + " bytes failed");
    scratch_bytes_ = b;
  }
  return static_cast<char*>(scratch_);
}

transport::Pair* Context::getPair(int peer) {
  if (peer < 0 || peer >= size || !pairs_[peer])
    throw EnforceNotMet("missing connection between rank " + std::to_string(rank) +
                        " (this process) and rank " + std::to_string(peer));
  return pairs_[peer].get();
}

void Context::closeConnections() {
  for (auto& p : pairs_)
    if (p) p->close();
}

void Context::signalException(const std::string& msg) {
  for (auto& p : pairs_)
    if (p) p->abort(msg);
}

namespace {
int listen_on(const std::string& host, int* port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) throw IoException("socket: " + std::string(std::strerror(errno)));
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = 0;
  if (::inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1)
    throw IoException("bad IPv4 address " + host);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd, 64) != 0)
    throw IoException("bind/listen: " + std::string(std::strerror(errno)));
  socklen_t len = sizeof(a);
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
  *port = ntohs(a.sin_port);
  return fd;
}

int connect_to(const std::string& host, int port) {
  for (int attempt = 0; attempt < 200; attempt++) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    ::inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) return fd;
    ::close(fd);
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  throw IoException("connect to " + host + ":" + std::to_string(port) + " failed");
}
}  // namespace

void Context::connectFullMesh(Store& store, const std::string& host, const std::string& prefix) {
  if (size == 1) return;
  int port = 0;
  int lfd = listen_on(host, &port);
  store.set(prefix + "_addr_" + std::to_string(rank), host + ":" + std::to_string(port));
  // rank r accepts from every higher rank and connects to every lower rank; the connecting
  // side announces its rank in the first 4 bytes
  for (int peer = 0; peer < rank; peer++) {
    const std::string v = store.get(prefix + "_addr_" + std::to_string(peer), timeout_);
    const auto colon = v.rfind(':');
    int fd = connect_to(v.substr(0, colon), std::stoi(v.substr(colon + 1)));
    int32_t me = rank;
    if (::send(fd, &me, sizeof(me), 0) != sizeof(me)) throw IoException("handshake send");
    pairs_[peer].reset(new transport::Pair(fd, rank, peer));
  }
  for (int k = rank + 1; k < size; k++) {
    int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) throw IoException("accept: " + std::string(std::strerror(errno)));
    int32_t who = -1;
    if (::recv(fd, &who, sizeof(who), MSG_WAITALL) != sizeof(who) || who <= rank || who >= size)
      throw IoException("handshake recv");
    pairs_[who].reset(new transport::Pair(fd, rank, who));
  }
  ::close(lfd);
}

// ---- unbound buffer -------------------------------------------------------------------------
UnboundBuffer::~UnboundBuffer() = default;

void UnboundBuffer::send(int dst, uint64_t slot, size_t offset, size_t nbytes) {
  if (offset + nbytes > size) throw EnforceNotMet("send out of buffer range");
  auto op = std::make_shared<Op>();
  op->ptr = static_cast<char*>(ptr) + offset;
  op->nbytes = nbytes;
  op->slot = slot;
  {
    std::lock_guard<std::mutex> g(mu_);
    sends_.push_back(op);
  }
  ctx_->getPair(dst)->postSend(op);
}

void UnboundBuffer::recv(int src, uint64_t slot, size_t offset, size_t nbytes) {
  if (offset + nbytes > size) throw EnforceNotMet("recv out of buffer range");
  auto op = std::make_shared<Op>();
  op->ptr = static_cast<char*>(ptr) + offset;
  op->nbytes = nbytes;
  op->slot = slot;
  {
    std::lock_guard<std::mutex> g(mu_);
    recvs_.push_back(op);
  }
  ctx_->getPair(src)->postRecv(op);
}

namespace {
void wait_oldest(Context* ctx, std::mutex& mu, std::vector<std::shared_ptr<UnboundBuffer::Op>>& q,
                 std::chrono::milliseconds timeout, const char* what) {
  std::shared_ptr<UnboundBuffer::Op> op;
  {
    std::lock_guard<std::mutex> g(mu);
    if (q.empty()) throw EnforceNotMet(std::string("no pending ") + what + " operation");
    op = q.front();
  }
  std::string timed_out, failed;
  {
    std::unique_lock<std::mutex> l(op->mu);
    // system_clock deadline: lowers to pthread_cond_timedwait (steady_clock's
    // pthread_cond_clockwait is invisible to GCC 11's ThreadSanitizer)
    const auto deadline = std::chrono::system_clock::now() + timeout;
    if (!op->cv.wait_until(l, deadline, [&] { return op->done; }))
      // the reference's message (gloo/gloo/transport/tcp/unbound_buffer.cc:80-84)
      timed_out = "Timed out waiting " + std::to_string(timeout.count()) + "ms for " + what +
                  " operation to complete";
    else if (!op->error.empty())
      failed = op->error;
  }
  {
    std::lock_guard<std::mutex> g(mu);
    q.erase(q.begin());
  }
  if (!timed_out.empty()) {
    // the op may still sit in a pair's queue, pointing into the caller's memory: poison the
    // context (every pair fails and joins its threads) before the exception unwinds that
    // memory, as the reference signals the context (tcp/unbound_buffer.cc:66-76)
    ctx->signalException(timed_out);
    throw IoException(timed_out);
  }
  if (!failed.empty()) throw IoException(failed);
}
}  // namespace

void UnboundBuffer::waitSend(std::chrono::milliseconds timeout) {
  wait_oldest(ctx_, mu_, sends_, timeout, "send");
}

void UnboundBuffer::waitRecv(std::chrono::milliseconds timeout) {
  wait_oldest(ctx_, mu_, recvs_, timeout, "recv");
}

}  // namespace hydra

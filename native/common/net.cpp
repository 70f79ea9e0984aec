// Implementation of net.h (see header).
#include "net.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/sha.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <signal.h>
#include <stdarg.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <fstream>
#include <sstream>

namespace dsa {

// ---------------------------------------------------------------------------------------------
// logging
// ---------------------------------------------------------------------------------------------
static std::atomic<int> g_log_level{LOG_INFO};
static std::mutex g_log_mu;

void set_log_level(int level) { g_log_level = level; }
int log_level() { return g_log_level; }

void logf(int level, const char* fmt, ...) {
  if (level > g_log_level) return;
  static const char* names[] = {"", "", "ERROR", "WARN", "INFO", "DEBUG", "TRACE"};
  char ts[64];
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  struct tm tmv;
  gmtime_r(&tv.tv_sec, &tmv);
  snprintf(ts, sizeof ts, "%04d-%02d-%02dT%02d:%02d:%02d.%03ldZ", tmv.tm_year + 1900, tmv.tm_mon + 1,
           tmv.tm_mday, tmv.tm_hour, tmv.tm_min, tmv.tm_sec, (long)(tv.tv_usec / 1000));
  char msg[4096];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof msg, fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(g_log_mu);
  fprintf(stderr, "%s %-5s %s\n", ts, names[level < 7 ? level : 6], msg);
  fflush(stderr);
}

// ---------------------------------------------------------------------------------------------
// utils
// ---------------------------------------------------------------------------------------------
static const char* B64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const std::string& in) {
  std::string out;
  out.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  while (i + 2 < in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    out.push_back(B64[(v >> 18) & 63]);
    out.push_back(B64[(v >> 12) & 63]);
    out.push_back(B64[(v >> 6) & 63]);
    out.push_back(B64[v & 63]);
    i += 3;
  }
  if (i + 1 == in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16);
    out.push_back(B64[(v >> 18) & 63]);
    out.push_back(B64[(v >> 12) & 63]);
    out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    out.push_back(B64[(v >> 18) & 63]);
    out.push_back(B64[(v >> 12) & 63]);
    out.push_back(B64[(v >> 6) & 63]);
    out.push_back('=');
  }
  return out;
}

std::string base64_decode(const std::string& in) {
  int T[256];
  for (int k = 0; k < 256; ++k) T[k] = -1;
  for (int k = 0; k < 64; ++k) T[(uint8_t)B64[k]] = k;
  T[(uint8_t)'-'] = 62;
  T[(uint8_t)'_'] = 63;
  std::string out;
  uint32_t v = 0;
  int bits = -8;
  for (unsigned char c : in) {
    if (T[c] < 0) continue;
    v = (v << 6) | T[c];
    bits += 6;
    if (bits >= 0) {
      out.push_back((char)((v >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return out;
}

int64_t now_micros() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}
int64_t now_millis() { return now_micros() / 1000; }

std::string url_decode(const std::string& s) {
  auto hex = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    // a '%' not followed by two hex digits is kept literally instead of throwing from a request thread
    if (s[i] == '%' && i + 2 < s.size() && hex(s[i + 1]) >= 0 && hex(s[i + 2]) >= 0) {
      out.push_back((char)(hex(s[i + 1]) * 16 + hex(s[i + 2])));
      i += 2;
    } else if (s[i] == '+') {
      out.push_back(' ');
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

std::string to_lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

bool write_file(const std::string& path, const std::string& data, int mode) {
  std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    if (!f) return false;
    f << data;
  }
  chmod(tmp.c_str(), mode);
  return rename(tmp.c_str(), path.c_str()) == 0;
}

bool mkdirs(const std::string& path, int mode) {
  if (path.empty()) return false;
  std::string cur;
  for (auto& part : split(path, '/')) {
    if (part.empty()) {
      if (cur.empty()) cur = "/";
      continue;
    }
    if (!cur.empty() && cur.back() != '/') cur.push_back('/');
    cur += part;
    if (mkdir(cur.c_str(), mode) != 0 && errno != EEXIST) return false;
  }
  return true;
}

bool path_exists(const std::string& path) {
  struct stat st;
  return stat(path.c_str(), &st) == 0;
}

// ---------------------------------------------------------------------------------------------
// request / response helpers
// ---------------------------------------------------------------------------------------------
std::string HttpRequest::header(const std::string& k, const std::string& def) const {
  auto it = headers.find(to_lower(k));
  return it == headers.end() ? def : it->second;
}
std::string HttpRequest::q(const std::string& k, const std::string& def) const {
  auto it = query.find(k);
  return it == query.end() ? def : it->second;
}
Json HttpRequest::json() const { return body.empty() ? Json::object() : Json::parse(body); }

HttpResponse HttpResponse::json(const Json& j, int status) {
  HttpResponse r;
  r.status = status;
  r.headers["Content-Type"] = "application/json";
  r.body = j.dump();
  return r;
}
HttpResponse HttpResponse::text(const std::string& t, int status) {
  HttpResponse r;
  r.status = status;
  r.headers["Content-Type"] = "text/plain";
  r.body = t;
  return r;
}
HttpResponse HttpResponse::error(int status, const std::string& msg) {
  Json j = Json::object();
  j.set("error", msg);
  return json(j, status);
}

static const char* status_text(int s) {
  switch (s) {
    case 101: return "Switching Protocols";
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

static bool send_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

// buffered reader over a socket
struct SockReader {
  int fd;
  std::string buf;
  size_t pos = 0;
  int timeout_ms;
  SSL* ssl = nullptr;
  bool fill() {
    if (pos > 0 && pos == buf.size()) {
      buf.clear();
      pos = 0;
    }
    char tmp[65536];
    if (ssl) {
      // TLS: records already decrypted inside OpenSSL need no poll; otherwise wait for bytes
      while (true) {
        if (SSL_pending(ssl) == 0) {
          struct pollfd p{fd, POLLIN, 0};
          if (::poll(&p, 1, timeout_ms) <= 0) return false;
        }
        int n = SSL_read(ssl, tmp, (int)sizeof tmp);
        if (n > 0) {
          buf.append(tmp, (size_t)n);
          return true;
        }
        int e = SSL_get_error(ssl, n);
        if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) return false;
      }
    }
    struct pollfd p{fd, POLLIN, 0};
    int r = ::poll(&p, 1, timeout_ms);
    if (r <= 0) return false;
    ssize_t n = ::recv(fd, tmp, sizeof tmp, 0);
    if (n <= 0) return false;
    buf.append(tmp, (size_t)n);
    return true;
  }
  bool read_line(std::string& line) {
    while (true) {
      size_t e = buf.find("\r\n", pos);
      if (e != std::string::npos) {
        line = buf.substr(pos, e - pos);
        pos = e + 2;
        return true;
      }
      if (buf.size() - pos > 1 << 20) return false;
      if (!fill()) return false;
    }
  }
  bool read_n(size_t n, std::string& out) {
    while (buf.size() - pos < n)
      if (!fill()) return false;
    out = buf.substr(pos, n);
    pos += n;
    return true;
  }
  bool read_some(std::string& out) {
    if (buf.size() == pos && !fill()) return false;
    out = buf.substr(pos);
    pos = buf.size();
    return true;
  }
};

// ---------------------------------------------------------------------------------------------
// WebSocket (server side, RFC 6455; unmasked frames from server)
// ---------------------------------------------------------------------------------------------
bool WsConn::send_frame(int opcode, const std::string& data) {
  std::lock_guard<std::mutex> lk(mu_);
  if (closed_) return false;
  std::string h;
  h.push_back((char)(0x80 | opcode));
  size_t n = data.size();
  if (n < 126) {
    h.push_back((char)n);
  } else if (n < 65536) {
    h.push_back((char)126);
    h.push_back((char)((n >> 8) & 0xFF));
    h.push_back((char)(n & 0xFF));
  } else {
    h.push_back((char)127);
    for (int k = 7; k >= 0; --k) h.push_back((char)((n >> (8 * k)) & 0xFF));
  }
  if (!send_all(fd_, h.data(), h.size()) || !send_all(fd_, data.data(), data.size())) {
    closed_ = true;
    return false;
  }
  return true;
}

void WsConn::close(int code) {
  std::string payload;
  payload.push_back((char)((code >> 8) & 0xFF));
  payload.push_back((char)(code & 0xFF));
  send_frame(0x8, payload);
  std::lock_guard<std::mutex> lk(mu_);
  closed_ = true;
}

bool WsConn::poll_peer(int timeout_ms) {
  if (closed_) return false;
  struct pollfd p{fd_, POLLIN, 0};
  int r = ::poll(&p, 1, timeout_ms);
  if (r <= 0) return true;  // nothing from the peer
  char buf[4096];
  ssize_t n = ::recv(fd_, buf, sizeof buf, MSG_DONTWAIT);
  if (n <= 0) {
    closed_ = true;
    return false;
  }
  // a close frame from the client (opcode 8) ends the stream; other frames are ignored
  if ((buf[0] & 0x0F) == 0x8) {
    closed_ = true;
    return false;
  }
  return true;
}

static std::string ws_accept_key(const std::string& key) {
  std::string s = key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
  unsigned char dig[SHA_DIGEST_LENGTH];
  SHA1((const unsigned char*)s.data(), s.size(), dig);
  return base64_encode(std::string((const char*)dig, SHA_DIGEST_LENGTH));
}

// ---------------------------------------------------------------------------------------------
// server
// ---------------------------------------------------------------------------------------------
HttpServer::~HttpServer() {
  stop();
  const int fd = listen_fd_.exchange(-1);
  if (fd >= 0) ::close(fd);
}

static std::vector<std::string> path_parts(const std::string& p) {
  std::vector<std::string> out;
  for (auto& s : split(p, '/'))
    if (!s.empty()) out.push_back(s);
  return out;
}

void HttpServer::route(const std::string& method, const std::string& pattern, HttpHandler h) {
  routes_.push_back(Route{method, path_parts(pattern), std::move(h), nullptr});
}

void HttpServer::websocket(const std::string& pattern, WsHandler h) {
  routes_.push_back(Route{"WS", path_parts(pattern), nullptr, std::move(h)});
}

bool HttpServer::match(const Route& r, const std::string& path, std::map<std::string, std::string>& params) const {
  auto parts = path_parts(path);
  if (parts.size() != r.parts.size()) return false;
  for (size_t k = 0; k < parts.size(); ++k) {
    const auto& rp = r.parts[k];
    if (rp.size() > 2 && rp.front() == '{' && rp.back() == '}') {
      params[rp.substr(1, rp.size() - 2)] = url_decode(parts[k]);
    } else if (rp != parts[k]) {
      return false;
    }
  }
  return true;
}

int HttpServer::start() {
  signal(SIGPIPE, SIG_IGN);
  const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) return -1;
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  struct sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port_);
  if (inet_pton(AF_INET, host_.c_str(), &addr.sin_addr) != 1) addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd, (struct sockaddr*)&addr, sizeof addr) != 0) {
    LOGE("bind %s:%d failed: %s", host_.c_str(), port_, strerror(errno));
    ::close(lfd);
    return -1;
  }
  if (::listen(lfd, 128) != 0) {
    ::close(lfd);
    return -1;
  }
  socklen_t len = sizeof addr;
  getsockname(lfd, (struct sockaddr*)&addr, &len);
  port_ = ntohs(addr.sin_port);
  listen_fd_ = lfd;
  running_ = true;
  return port_;
}

// The listening socket is owned by serve_forever() while it runs: stop() only flips running_ and
// shuts the socket down (waking poll/accept); the fd is closed by the serving thread on its way out
// (or by the destructor when it never served), so no thread closes an fd another is polling.
void HttpServer::serve_forever() {
  const int lfd = listen_fd_;
  while (running_) {
    struct pollfd p{lfd, POLLIN, 0};
    int r = ::poll(&p, 1, 200);
    if (r <= 0) continue;
    struct sockaddr_in caddr{};
    socklen_t clen = sizeof caddr;
    int fd = ::accept(lfd, (struct sockaddr*)&caddr, &clen);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    char ip[64];
    inet_ntop(AF_INET, &caddr.sin_addr, ip, sizeof ip);
    std::thread(&HttpServer::handle_conn, this, fd, std::string(ip)).detach();
  }
  int expected = lfd;
  if (listen_fd_.compare_exchange_strong(expected, -1)) ::close(lfd);
}

void HttpServer::stop() {
  running_ = false;
  const int fd = listen_fd_;
  if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
}

static void parse_query(const std::string& qs, std::map<std::string, std::string>& out) {
  for (auto& kv : split(qs, '&')) {
    if (kv.empty()) continue;
    auto eq = kv.find('=');
    if (eq == std::string::npos)
      out[url_decode(kv)] = "";
    else
      out[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
  }
}

// Content-Length is 1*DIGIT (RFC 9110 §8.6); anything else (sign, spaces, hex, overflow) is
// rejected rather than handed to stoull, whose exceptions would end the agent from a worker thread.
static bool parse_content_length(const std::string& v, size_t& out) {
  if (v.empty() || v.size() > 18) return false;
  size_t n = 0;
  for (char c : v) {
    if (c < '0' || c > '9') return false;
    n = n * 10 + (size_t)(c - '0');
  }
  out = n;
  return true;
}

static constexpr size_t kMaxHeaderBytes = 64 << 10;
static constexpr size_t kMaxHeaders = 128;
static constexpr size_t kMaxBody = (size_t)512 << 20;

static void send_error_and_close(int fd, int status, const char* msg) {
  auto r = HttpResponse::error(status, msg);
  std::string out = "HTTP/1.1 " + std::to_string(status) + " " + status_text(status) +
                    "\r\nContent-Length: " + std::to_string(r.body.size()) + "\r\nConnection: close\r\n\r\n" + r.body;
  send_all(fd, out.data(), out.size());
}

void HttpServer::handle_conn(int fd, std::string remote) {
  // A connection thread is detached: nothing may escape it, or std::terminate takes the whole
  // shim/runner down because of one bad client.
  try {
    serve_conn(fd, remote);
  } catch (const std::exception& e) {
    LOGW("connection from %s dropped: %s", remote.c_str(), e.what());
  } catch (...) {
    LOGW("connection from %s dropped", remote.c_str());
  }
  ::close(fd);
}

void HttpServer::serve_conn(int fd, const std::string& remote) {
  SockReader rd{fd, {}, 0, 120000};
  while (running_) {
    std::string line;
    if (!rd.read_line(line)) break;
    if (line.empty()) continue;
    HttpRequest req;
    req.remote_addr = remote;
    auto sp1 = line.find(' '), sp2 = line.rfind(' ');
    if (sp1 == std::string::npos || sp2 == sp1) break;
    req.method = line.substr(0, sp1);
    std::string target = line.substr(sp1 + 1, sp2 - sp1 - 1);
    auto qm = target.find('?');
    req.path = qm == std::string::npos ? target : target.substr(0, qm);
    if (qm != std::string::npos) parse_query(target.substr(qm + 1), req.query);
    bool bad = false, too_big = false;
    size_t header_bytes = 0, n_headers = 0;
    while (true) {
      if (!rd.read_line(line)) {
        bad = true;
        break;
      }
      if (line.empty()) break;
      header_bytes += line.size() + 2;
      if (++n_headers > kMaxHeaders || header_bytes > kMaxHeaderBytes) {
        too_big = true;
        break;
      }
      auto c = line.find(':');
      if (c != std::string::npos) req.headers[to_lower(trim(line.substr(0, c)))] = trim(line.substr(c + 1));
    }
    if (too_big) {
      send_error_and_close(fd, 431, "request headers too large");
      break;
    }
    if (bad) break;
    // Only Content-Length framed bodies: a chunked body would otherwise be read as the next request.
    if (!req.header("transfer-encoding").empty()) {
      send_error_and_close(fd, 411, "Transfer-Encoding not supported; send Content-Length");
      break;
    }
    size_t clen = 0;
    if (req.headers.count("content-length") && !parse_content_length(req.headers["content-length"], clen)) {
      send_error_and_close(fd, 400, "invalid Content-Length");
      break;
    }
    if (clen > kMaxBody) {
      send_error_and_close(fd, 413, "body too large");
      break;
    }
    if (clen > 0 && !rd.read_n(clen, req.body)) break;
    bool keep_alive = to_lower(req.header("connection")) != "close";

    // WebSocket upgrade
    if (to_lower(req.header("upgrade")) == "websocket") {
      for (auto& r : routes_) {
        if (r.method != "WS") continue;
        std::map<std::string, std::string> params;
        if (!match(r, req.path, params)) continue;
        req.params = params;
        std::string resp = "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                           "Sec-WebSocket-Accept: " +
                           ws_accept_key(req.header("sec-websocket-key")) + "\r\n\r\n";
        send_all(fd, resp.data(), resp.size());
        WsConn ws(fd);
        try {
          r.ws(req, ws);
        } catch (const std::exception& e) {
          LOGW("websocket handler error: %s", e.what());
        }
        if (!ws.closed()) ws.close();
        return;
      }
    }

    HttpResponse resp;
    bool found = false, method_mismatch = false;
    for (auto& r : routes_) {
      if (r.method == "WS") continue;
      std::map<std::string, std::string> params;
      if (!match(r, req.path, params)) continue;
      if (r.method != req.method) {
        method_mismatch = true;
        continue;
      }
      found = true;
      req.params = params;
      try {
        resp = r.handler(req);
      } catch (const std::exception& e) {
        resp = HttpResponse::error(500, e.what());
      }
      break;
    }
    if (!found) resp = method_mismatch ? HttpResponse::error(405, "method not allowed") : HttpResponse::error(404, "not found");
    LOGD("%s %s -> %d", req.method.c_str(), req.path.c_str(), resp.status);
    std::string out = "HTTP/1.1 " + std::to_string(resp.status) + " " + status_text(resp.status) + "\r\n";
    for (auto& h : resp.headers) out += h.first + ": " + h.second + "\r\n";
    out += "Content-Length: " + std::to_string(resp.body.size()) + "\r\n";
    out += keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
    out += resp.body;
    if (!send_all(fd, out.data(), out.size()) || !keep_alive) break;
  }
}

// ---------------------------------------------------------------------------------------------
// client
// ---------------------------------------------------------------------------------------------
static int connect_tcp(const std::string& host, int port, int timeout_ms, std::string& err) {
  struct addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    err = "resolve failed: " + host;
    return -1;
  }
  int fd = -1;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int r = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (r != 0 && errno == EINPROGRESS) {
      struct pollfd p{fd, POLLOUT, 0};
      if (::poll(&p, 1, timeout_ms) == 1) {
        int so = 0;
        socklen_t sl = sizeof so;
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl);
        r = so == 0 ? 0 : -1;
      } else {
        r = -1;
      }
    }
    if (r == 0) {
      fcntl(fd, F_SETFL, fl);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      break;
    }
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) err = "connect failed: " + host + ":" + std::to_string(port);
  return fd;
}

static int connect_unix(const std::string& path, std::string& err) {
  int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
  struct sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  strncpy(addr.sun_path, path.c_str(), sizeof(addr.sun_path) - 1);
  if (::connect(fd, (struct sockaddr*)&addr, sizeof addr) != 0) {
    err = "connect unix socket failed: " + path;
    ::close(fd);
    return -1;
  }
  return fd;
}

// ---- TLS (agent downloads from https:// URLs: S3, release servers) ----
// One client context per process: system CA store (or an explicit CA file), peer and hostname
// verification on, TLS 1.2+.  The handshake runs on the connected blocking socket.
struct TlsConn {
  SSL_CTX* ctx = nullptr;
  SSL* ssl = nullptr;
  ~TlsConn() {
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
    }
    if (ctx) SSL_CTX_free(ctx);
  }
};

static bool tls_connect(int fd, const HttpClientRequest& req, TlsConn& t, std::string& err) {
  t.ctx = SSL_CTX_new(TLS_client_method());
  if (!t.ctx) {
    err = "TLS: no context";
    return false;
  }
  SSL_CTX_set_min_proto_version(t.ctx, TLS1_2_VERSION);
  if (!req.insecure) {
    SSL_CTX_set_verify(t.ctx, SSL_VERIFY_PEER, nullptr);
    const char* env_ca = getenv("DSTACK_CA_FILE");
    const std::string ca = !req.ca_file.empty() ? req.ca_file : (env_ca ? env_ca : "");
    if (!ca.empty() ? SSL_CTX_load_verify_locations(t.ctx, ca.c_str(), nullptr) != 1
                    : SSL_CTX_set_default_verify_paths(t.ctx) != 1) {
      err = "TLS: cannot load CA certificates" + (ca.empty() ? std::string() : " from " + ca);
      return false;
    }
  }
  t.ssl = SSL_new(t.ctx);
  SSL_set_fd(t.ssl, fd);
  SSL_set_tlsext_host_name(t.ssl, req.host.c_str());  // SNI
  if (!req.insecure) SSL_set1_host(t.ssl, req.host.c_str());  // certificate must name the host
  if (SSL_connect(t.ssl) != 1) {
    long vr = SSL_get_verify_result(t.ssl);
    char ebuf[256];
    ERR_error_string_n(ERR_get_error(), ebuf, sizeof ebuf);
    err = std::string("TLS handshake with ") + req.host + " failed: " +
          (vr != X509_V_OK ? X509_verify_cert_error_string(vr) : ebuf);
    return false;
  }
  return true;
}

static bool tls_send_all(SSL* ssl, const char* p, size_t n) {
  while (n > 0) {
    int w = SSL_write(ssl, p, (int)std::min<size_t>(n, 1 << 30));
    if (w <= 0) return false;
    p += w;
    n -= (size_t)w;
  }
  return true;
}

HttpClientResponse http_request(const HttpClientRequest& req) {
  HttpClientResponse resp;
  int fd = req.unix_socket.empty() ? connect_tcp(req.host, req.port, req.timeout_ms, resp.error)
                                   : connect_unix(req.unix_socket, resp.error);
  if (fd < 0) return resp;
  TlsConn tls;
  if (req.tls) {
    // bounded handshake: the socket is blocking, so give it the request's timeout
    struct timeval tv{req.timeout_ms / 1000, (req.timeout_ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (!tls_connect(fd, req, tls, resp.error)) {
      ::close(fd);
      return resp;
    }
  }
  std::string out = req.method + " " + req.path + " HTTP/1.1\r\n";
  const bool default_port = req.port == (req.tls ? 443 : 80);
  out += "Host: " + (req.unix_socket.empty() ? req.host + (default_port ? "" : ":" + std::to_string(req.port))
                                             : std::string("docker")) + "\r\n";
  bool has_ct = false;
  for (auto& h : req.headers) {
    out += h.first + ": " + h.second + "\r\n";
    if (to_lower(h.first) == "content-type") has_ct = true;
  }
  if (!req.body.empty() && !has_ct) out += "Content-Type: application/json\r\n";
  out += "Content-Length: " + std::to_string(req.body.size()) + "\r\nConnection: close\r\n\r\n";
  out += req.body;
  if (!(tls.ssl ? tls_send_all(tls.ssl, out.data(), out.size()) : send_all(fd, out.data(), out.size()))) {
    resp.error = "send failed";
    ::close(fd);
    return resp;
  }
  SockReader rd{fd, {}, 0, req.timeout_ms};
  rd.ssl = tls.ssl;
  std::string line;
  if (!rd.read_line(line)) {
    resp.error = "no response";
    ::close(fd);
    return resp;
  }
  auto sp = line.find(' ');
  resp.status = sp == std::string::npos ? 0 : atoi(line.c_str() + sp + 1);
  while (rd.read_line(line) && !line.empty()) {
    auto c = line.find(':');
    if (c != std::string::npos) resp.headers[to_lower(trim(line.substr(0, c)))] = trim(line.substr(c + 1));
  }
  auto emit = [&](const std::string& chunk) -> bool {
    if (req.on_chunk) return req.on_chunk(chunk);
    resp.body += chunk;
    return true;
  };
  if (to_lower(resp.headers["transfer-encoding"]).find("chunked") != std::string::npos) {
    while (rd.read_line(line)) {
      char* end = nullptr;
      unsigned long long n = strtoull(line.c_str(), &end, 16);
      if (end == line.c_str()) {  // not a chunk-size line
        resp.error = "malformed chunked body";
        break;
      }
      if (n == 0) break;
      if (n > kMaxBody) {
        resp.error = "chunk too large";
        break;
      }
      std::string chunk;
      if (!rd.read_n((size_t)n, chunk)) break;
      if (!emit(chunk)) break;
      rd.read_line(line);  // CRLF after chunk
    }
  } else if (resp.headers.count("content-length")) {
    size_t n = 0;
    std::string body;
    if (!parse_content_length(resp.headers["content-length"], n) || n > kMaxBody)
      resp.error = "invalid Content-Length";
    else if (n > 0 && rd.read_n(n, body))
      emit(body);
  } else if (resp.status != 204 && resp.status != 101) {
    std::string chunk;
    while (rd.read_some(chunk))
      if (!emit(chunk)) break;
  }
  if (tls.ssl) {
    SSL_shutdown(tls.ssl);
    SSL_free(tls.ssl);
    tls.ssl = nullptr;
  }
  ::close(fd);
  if (!resp.error.empty()) resp.status = 0;  // body framing broken: treat as a transport error
  return resp;
}

bool parse_url(const std::string& url, HttpClientRequest& req) {
  std::string u = url;
  if (u.rfind("https://", 0) == 0) {
    req.tls = true;
    u = u.substr(8);
  } else if (u.rfind("http://", 0) == 0) {
    req.tls = false;
    u = u.substr(7);
  } else {
    return false;
  }
  auto slash = u.find('/');
  std::string hostport = slash == std::string::npos ? u : u.substr(0, slash);
  req.path = slash == std::string::npos ? "/" : u.substr(slash);
  auto colon = hostport.find(':');
  req.host = colon == std::string::npos ? hostport : hostport.substr(0, colon);
  req.port = colon == std::string::npos ? (req.tls ? 443 : 80) : atoi(hostport.c_str() + colon + 1);
  return !req.host.empty();
}

HttpClientResponse http_get_url(const std::string& url, int timeout_ms, const std::string& ca_file) {
  std::string cur = url;
  // follow redirects (release servers and S3 pre-signed URLs answer 301/302/307 with Location)
  for (int hop = 0; hop < 5; ++hop) {
    HttpClientRequest req;
    req.timeout_ms = timeout_ms;
    req.ca_file = ca_file;
    if (!parse_url(cur, req)) {
      HttpClientResponse r;
      r.error = "unsupported URL: " + cur;
      return r;
    }
    auto r = http_request(req);
    if ((r.status == 301 || r.status == 302 || r.status == 303 || r.status == 307 || r.status == 308) &&
        r.headers.count("location")) {
      std::string loc = r.headers["location"];
      if (loc.rfind("http", 0) != 0)  // relative: same scheme, host and port
        loc = std::string(req.tls ? "https://" : "http://") + req.host + ":" + std::to_string(req.port) + loc;
      cur = loc;
      continue;
    }
    return r;
  }
  HttpClientResponse r;
  r.error = "too many redirects";
  return r;
}

}  // namespace dsa

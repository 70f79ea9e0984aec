// Minimal HTTP/1.1 server + client + WebSocket for the dstack-amd native agents (C++17, POSIX).
//
// Server: one listener thread, one detached worker thread per connection (keep-alive), a router
// with {param} path segments, and an in-place upgrade to WebSocket for streaming logs.
// Client: TCP, TLS (OpenSSL, verified) or unix-socket (Docker Engine API), Content-Length and chunked
// bodies, optional streaming callback for long-lived chunked responses (image pull progress).
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "json.h"

namespace dsa {

// ---------------------------------------------------------------------------------------------
// logging
// ---------------------------------------------------------------------------------------------
enum LogLevel { LOG_ERROR = 2, LOG_WARN = 3, LOG_INFO = 4, LOG_DEBUG = 5, LOG_TRACE = 6 };
void set_log_level(int level);
int log_level();
void logf(int level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#define LOGE(...) ::dsa::logf(::dsa::LOG_ERROR, __VA_ARGS__)
#define LOGW(...) ::dsa::logf(::dsa::LOG_WARN, __VA_ARGS__)
#define LOGI(...) ::dsa::logf(::dsa::LOG_INFO, __VA_ARGS__)
#define LOGD(...) ::dsa::logf(::dsa::LOG_DEBUG, __VA_ARGS__)

// ---------------------------------------------------------------------------------------------
// small utils
// ---------------------------------------------------------------------------------------------
std::string base64_encode(const std::string& in);
std::string base64_decode(const std::string& in);
int64_t now_micros();
int64_t now_millis();
std::string url_decode(const std::string& s);
std::string to_lower(std::string s);
std::vector<std::string> split(const std::string& s, char sep);
std::string trim(const std::string& s);
bool read_file(const std::string& path, std::string& out);
bool write_file(const std::string& path, const std::string& data, int mode = 0644);
bool mkdirs(const std::string& path, int mode = 0755);
bool path_exists(const std::string& path);

// ---------------------------------------------------------------------------------------------
// HTTP server
// ---------------------------------------------------------------------------------------------
struct HttpRequest {
  std::string method;
  std::string path;
  std::map<std::string, std::string> query;
  std::map<std::string, std::string> headers;  // lower-case keys
  std::map<std::string, std::string> params;   // from {param} route segments
  std::string body;
  std::string remote_addr;

  std::string header(const std::string& k, const std::string& def = "") const;
  std::string q(const std::string& k, const std::string& def = "") const;
  Json json() const;  // throws on invalid JSON
};

struct HttpResponse {
  int status = 200;
  std::map<std::string, std::string> headers;
  std::string body;

  static HttpResponse json(const Json& j, int status = 200);
  static HttpResponse text(const std::string& t, int status = 200);
  static HttpResponse error(int status, const std::string& msg);
};

class WsConn {
 public:
  explicit WsConn(int fd) : fd_(fd) {}
  bool send_text(const std::string& data) { return send_frame(0x1, data); }
  bool send_binary(const std::string& data) { return send_frame(0x2, data); }
  void close(int code = 1000);
  bool closed() const { return closed_; }
  // non-blocking check for a close/ping from the peer; returns false once the peer has gone
  bool poll_peer(int timeout_ms);

 private:
  bool send_frame(int opcode, const std::string& data);
  int fd_;
  bool closed_ = false;
  std::mutex mu_;
};

using HttpHandler = std::function<HttpResponse(HttpRequest&)>;
using WsHandler = std::function<void(HttpRequest&, WsConn&)>;

class HttpServer {
 public:
  HttpServer(std::string host, int port) : host_(std::move(host)), port_(port) {}
  ~HttpServer();
  void route(const std::string& method, const std::string& pattern, HttpHandler h);
  void websocket(const std::string& pattern, WsHandler h);
  // bind + listen; returns the bound port (useful with port 0) or -1
  int start();
  void serve_forever();  // blocks until stop()
  void stop();
  int port() const { return port_; }

 private:
  struct Route {
    std::string method;
    std::vector<std::string> parts;
    HttpHandler handler;
    WsHandler ws;
  };
  bool match(const Route& r, const std::string& path, std::map<std::string, std::string>& params) const;
  void handle_conn(int fd, std::string remote);
  void serve_conn(int fd, const std::string& remote);
  std::string host_;
  int port_;
  std::atomic<int> listen_fd_{-1};
  std::atomic<bool> running_{false};
  std::vector<Route> routes_;
};

// ---------------------------------------------------------------------------------------------
// HTTP client
// ---------------------------------------------------------------------------------------------
struct HttpClientResponse {
  int status = 0;  // 0 = transport error
  std::map<std::string, std::string> headers;
  std::string body;
  std::string error;
  bool ok() const { return status >= 200 && status < 300; }
};

struct HttpClientRequest {
  std::string method = "GET";
  std::string host = "127.0.0.1";
  int port = 80;
  std::string unix_socket;  // if set, connect here instead of host:port
  std::string path = "/";
  std::map<std::string, std::string> headers;
  std::string body;
  int timeout_ms = 30000;
  // streaming: called with each decoded body chunk; return false to abort
  std::function<bool(const std::string&)> on_chunk;
  // TLS (https): verified against the system CA store, or ca_file / $DSTACK_CA_FILE; the
  // certificate must name `host` (SNI + hostname check).  insecure skips verification.
  bool tls = false;
  std::string ca_file;
  bool insecure = false;
};

HttpClientResponse http_request(const HttpClientRequest& req);
// "http[s]://host[:port]/path" -> host, port, path, tls
bool parse_url(const std::string& url, HttpClientRequest& req);
// GET http:// or https:// URL, following up to 5 redirects
HttpClientResponse http_get_url(const std::string& url, int timeout_ms = 30000, const std::string& ca_file = "");

}  // namespace dsa

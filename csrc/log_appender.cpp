// Rotating log file appender with its own writer thread (the node's app.log).
//
// reference: upow/my_logger.py:8-53 — a RotatingFileHandler on logs/app.log (5 MB x 100 files, DEBUG).
// The node logs a line per /push_tx, so at a four-digit tx rate the Python logging machinery on a
// listener thread (format, shouldRollover's os.path checks, write, flush per record) competes with the
// HTTP event loop for the GIL. Here a record costs the caller one mutex-protected append of the finished
// line; a C++ thread writes the buffered lines, and rotates the files (app.log -> app.log.1 -> ... ->
// app.log.<backups>) when the next write would pass max_bytes, as RotatingFileHandler does.
//
// Bounded: at most `max_pending` bytes wait for the writer (a stalled stderr pipe or disk must not grow the
// node's memory); past that, lines are dropped and counted, and the writer notes the count in the log once
// it catches up. An urgent record (ERROR and above) is written before the call returns, so the last lines
// before an abort are not left in the buffer.
#include <pybind11/pybind11.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace upow {
namespace {

class LogAppender {
public:
    LogAppender(std::string path, int64_t max_bytes, int backups)
        : path_(std::move(path)), max_bytes_(max_bytes), backups_(backups) {
        open_file();
        thread_ = std::thread([this] { run(); });
    }
    // an already open descriptor (the process's stderr, dup'ed: its file offset is shared, so lines never
    // overwrite what other code writes to fd 2); no rotation
    explicit LogAppender(int fd) : max_bytes_(0), backups_(0), fd_(fd) {
        if (fd_ < 0) throw std::runtime_error("log appender: bad descriptor");
        thread_ = std::thread([this] { run(); });
    }
    ~LogAppender() { close(); }

    // returns false when the line was dropped (buffer full)
    bool write(const char* p, size_t n, bool urgent = false) {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (closed_) return false;
            if (!urgent && pending_.size() + n > max_pending_) {  // urgent records are never dropped
                ++dropped_;
                ++dropped_unreported_;
                return false;
            }
            pending_.append(p, n);
            ++records_;
        }
        // no wake-up: the writer thread drains every 20 ms (a flush or close wakes it at once)
        return true;
    }

    // an urgent record: appended, then written before returning (the caller released the GIL); a writer
    // stuck on a stalled pipe costs the caller at most 100 ms, never a hang
    void write_sync(const std::string& line) {
        if (write(line.data(), line.size(), true)) flush_for(100);
    }

    void set_max_pending(int64_t n) {
        std::lock_guard<std::mutex> g(mu_);
        max_pending_ = size_t(std::max<int64_t>(4096, n));
    }

    int64_t dropped() {
        std::lock_guard<std::mutex> g(mu_);
        return int64_t(dropped_);
    }

    // everything written so far is in the file (tests, shutdown)
    void flush() { flush_for(-1); }

    // flush, waiting at most `ms` milliseconds (< 0: until done); true when everything is written
    bool flush_for(int64_t ms) {
        std::unique_lock<std::mutex> lk(mu_);
        const uint64_t want = records_;
        ++flush_req_;
        cv_.notify_one();
        auto done = [&] { return written_records_ >= want || closed_; };
        if (ms < 0) {
            done_cv_.wait(lk, done);
            return true;
        }
        return done_cv_.wait_for(lk, std::chrono::milliseconds(ms), done);
    }

    void close() {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (stop_) return;
            stop_ = true;
        }
        cv_.notify_one();
        if (thread_.joinable()) thread_.join();
        std::lock_guard<std::mutex> g(mu_);
        closed_ = true;
        if (fd_ >= 0) ::close(fd_);
        fd_ = -1;
        done_cv_.notify_all();
    }

    int64_t rotations() {
        std::lock_guard<std::mutex> g(mu_);
        return rotations_;
    }

private:
    void open_file() {
        fd_ = ::open(path_.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
        if (fd_ < 0) throw std::runtime_error("log appender: cannot open " + path_ + ": " + std::strerror(errno));
        const off_t end = ::lseek(fd_, 0, SEEK_END);
        size_ = end > 0 ? int64_t(end) : 0;
    }

    void rotate() {
        ::close(fd_);
        fd_ = -1;
        if (backups_ > 0) {
            for (int i = backups_ - 1; i >= 1; --i) {
                const std::string src = path_ + "." + std::to_string(i), dst = path_ + "." + std::to_string(i + 1);
                ::rename(src.c_str(), dst.c_str());  // missing sources are fine
            }
            ::rename(path_.c_str(), (path_ + ".1").c_str());
        } else {
            ::unlink(path_.c_str());
        }
        ++rotations_;
        open_file();
    }

    void write_all(const char* p, size_t n) {
        while (n) {
            const ssize_t w = ::write(fd_, p, n);
            if (w < 0) {
                if (errno == EINTR) continue;
                return;  // a full disk must not take the node down: the line is dropped
            }
            p += w;
            n -= size_t(w);
        }
    }

    // line by line so a rotation lands between records, as RotatingFileHandler's does
    void drain(const std::string& buf) {
        size_t at = 0;
        while (at < buf.size()) {
            size_t nl = buf.find('\n', at);
            const size_t end = nl == std::string::npos ? buf.size() : nl + 1;
            const size_t len = end - at;
            if (max_bytes_ > 0 && size_ > 0 && size_ + int64_t(len) >= max_bytes_) rotate();
            if (fd_ >= 0) write_all(buf.data() + at, len);
            size_ += int64_t(len);
            at = end;
        }
    }

    void run() {
        std::string buf;
        for (;;) {
            uint64_t taken, lost = 0;
            {
                std::unique_lock<std::mutex> lk(mu_);
                // batch: wake on data, but give a burst ~20 ms to accumulate unless someone waits on a flush
                cv_.wait_for(lk, std::chrono::milliseconds(20), [&] { return stop_ || flush_req_ != flush_seen_; });
                flush_seen_ = flush_req_;
                buf.swap(pending_);
                taken = records_;
                std::swap(lost, dropped_unreported_);
                if (buf.empty() && stop_) {
                    written_records_ = taken;
                    done_cv_.notify_all();
                    return;
                }
            }
            if (!buf.empty()) drain(buf);
            if (lost) {
                const std::string note = "log appender: " + std::to_string(lost) + " line(s) dropped (buffer full)\n";
                drain(note);
            }
            buf.clear();
            {
                std::lock_guard<std::mutex> g(mu_);
                written_records_ = taken;
            }
            done_cv_.notify_all();
        }
    }

    std::string path_;
    int64_t max_bytes_;
    int backups_;
    int fd_ = -1;
    int64_t size_ = 0, rotations_ = 0;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::string pending_;
    size_t max_pending_ = size_t(8) << 20;
    uint64_t records_ = 0, written_records_ = 0, flush_req_ = 0, flush_seen_ = 0, dropped_ = 0, dropped_unreported_ = 0;
    bool stop_ = false, closed_ = false;
    std::thread thread_;
};

}  // namespace

void register_log_appender(py::module_& m) {
    py::class_<LogAppender>(m, "LogAppender")
        .def(py::init<std::string, int64_t, int>(), py::arg("path"), py::arg("max_bytes"), py::arg("backups"))
        .def(py::init<int>(), py::arg("fd"))
        .def("write",
             [](LogAppender& a, py::str s) {
                 Py_ssize_t n = 0;
                 const char* p = PyUnicode_AsUTF8AndSize(s.ptr(), &n);
                 if (!p) throw py::error_already_set();
                 return a.write(p, size_t(n), false);
             })
        .def("write_sync",
             [](LogAppender& a, py::str s) {
                 std::string line = s;
                 py::gil_scoped_release nogil;
                 a.write_sync(line);
             })
        .def("set_max_pending", &LogAppender::set_max_pending, py::arg("bytes"))
        .def_property_readonly("dropped", &LogAppender::dropped)
        .def("flush", &LogAppender::flush, py::call_guard<py::gil_scoped_release>())
        .def("close", &LogAppender::close, py::call_guard<py::gil_scoped_release>())
        .def_property_readonly("rotations", &LogAppender::rotations);
}

}  // namespace upow

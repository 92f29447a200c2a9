// Native stall probe: what every thread of this process is doing while the HTTP event loop is late.
//
// The node's Python watchdog (node/main.py _loop_lag_monitor) samples stacks with sys._current_frames(),
// which needs the GIL: a stall in which one thread holds the GIL (or the whole process waits in the kernel)
// leaves it with no sample at all. This probe is a plain C++ thread that never touches Python: every
// `period_us` it reads the loop's heartbeat (a float64 the loop stores as time.perf_counter(), i.e.
// CLOCK_MONOTONIC) and, while the heartbeat is older than `late_ms`, appends one JSON line per sample:
// the wall time, how late the loop is, and for the loop thread plus every thread that is running (R) or in
// uninterruptible sleep (D): tid, comm, state, kernel wait channel and current syscall number
// (/proc/<pid>/task/<tid>/{stat,wchan,syscall}). The node maps tids to Python thread names (<trace>.threads).
#include <pybind11/pybind11.h>

#include <dirent.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <memory>
#include <string>
#include <thread>

namespace py = pybind11;

namespace {

std::string read_small(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return {};
    char buf[512];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    std::string s(buf, n);
    while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
    return s;
}

std::string json_escape(const std::string& s) {
    std::string o;
    for (char c : s) {
        if (c == '"' || c == '\\') o += '\\';
        if (static_cast<unsigned char>(c) < 0x20) continue;
        o += c;
    }
    return o;
}

class StallProbe {
public:
    // heartbeat None: sample on every period (`pid`: another process, e.g. the node a soak script started --
    // a process-wide freeze of the node then does not freeze its observer). Samples are kept in memory and
    // written at stop(): a probe that wrote each one could itself wait in the kernel's dirty-page throttling,
    // the very kind of stall it is there to see.
    StallProbe(std::string path, py::object heartbeat, long loop_tid, double late_ms, int period_us, long pid)
        : path_(std::move(path)), loop_tid_(loop_tid), late_s_(late_ms / 1000.0), period_us_(period_us),
          task_dir_(pid > 0 ? "/proc/" + std::to_string(pid) + "/task" : std::string("/proc/self/task")) {
        if (!heartbeat.is_none()) {
            py::buffer_info bi = heartbeat.cast<py::buffer>().request(true);
            if (bi.itemsize != 8 || bi.size < 1 || bi.format != py::format_descriptor<double>::format())
                throw std::invalid_argument("heartbeat must be a writable float64 array of at least one element");
            hb_owner_ = heartbeat;  // keeps the array alive while the probe reads it
            hb_ = static_cast<volatile double*>(bi.ptr);
        }
        if (period_us < 200 || late_ms <= 0) throw std::invalid_argument("period_us >= 200 and late_ms > 0");
        out_ = std::fopen(path_.c_str(), "a");
        if (!out_) throw std::runtime_error("stall probe: cannot open " + path_);
        buf_.reserve(size_t(1) << 20);
        thread_ = std::thread([this] { run(); });
    }
    ~StallProbe() { stop(); }

    void stop() {
        if (stop_.exchange(true)) return;
        if (thread_.joinable()) thread_.join();
        if (out_) {
            std::fwrite(buf_.data(), 1, buf_.size(), out_);
            std::fclose(out_);
        }
        out_ = nullptr;
    }
    long samples() const { return samples_.load(); }

private:
    void run() {
        pthread_setname_np(pthread_self(), "upow-stallprobe");
        const long self = long(syscall(SYS_gettid));
        while (!stop_.load()) {
            std::this_thread::sleep_for(std::chrono::microseconds(period_us_));
            timespec ts{};
            clock_gettime(CLOCK_MONOTONIC, &ts);
            const double now = double(ts.tv_sec) + double(ts.tv_nsec) * 1e-9;
            const double late = hb_ ? now - *hb_ : 0.0;
            if (hb_ && !(late > late_s_)) continue;
            sample(late, self);
        }
    }

    void sample(double late, long self) {
        timespec wall{};
        clock_gettime(CLOCK_REALTIME, &wall);
        std::string line = "{\"t\": " + std::to_string(double(wall.tv_sec) + double(wall.tv_nsec) * 1e-9) +
                           ", \"late_ms\": " + std::to_string(late * 1000.0) + ", \"threads\": [";
        DIR* d = opendir(task_dir_.c_str());
        if (!d) return;
        bool first = true;
        while (dirent* e = readdir(d)) {
            if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
            const long tid = std::atol(e->d_name);
            if (tid == self) continue;
            const std::string base = task_dir_ + "/" + e->d_name;
            const std::string stat = read_small(base + "/stat");
            // "tid (comm) S ...": comm may hold spaces or parentheses, the state follows the last ')'
            const size_t rp = stat.rfind(')');
            if (rp == std::string::npos || rp + 2 >= stat.size()) continue;
            const char state = stat[rp + 2];
            if (tid != loop_tid_ && state != 'R' && state != 'D') continue;
            const size_t lp = stat.find('(');
            const std::string comm = lp == std::string::npos ? "" : stat.substr(lp + 1, rp - lp - 1);
            const std::string wchan = read_small(base + "/wchan");
            std::string sc = read_small(base + "/syscall");
            const size_t sp = sc.find(' ');
            if (sp != std::string::npos) sc.resize(sp);
            line += std::string(first ? "" : ", ") + "[" + std::to_string(tid) + ", \"" + json_escape(comm) + "\", \"" +
                    state + "\", \"" + json_escape(wchan) + "\", \"" + json_escape(sc) + "\"]";
            first = false;
        }
        closedir(d);
        line += "]}\n";
        if (buf_.size() + line.size() > kMaxBuf) return;  // bounded: the first kMaxBuf bytes of samples
        buf_ += line;
        ++samples_;
    }

    static constexpr size_t kMaxBuf = size_t(64) << 20;
    std::string path_;
    long loop_tid_;
    double late_s_;
    int period_us_;
    std::string task_dir_;
    std::string buf_;
    py::object hb_owner_;
    volatile double* hb_ = nullptr;
    FILE* out_ = nullptr;
    std::atomic<bool> stop_{false};
    std::atomic<long> samples_{0};
    std::thread thread_;
};

}  // namespace

namespace upow {

void register_stall_probe(py::module_& m) {
    py::class_<StallProbe>(m, "StallProbe")
        .def(py::init<std::string, py::object, long, double, int, long>(), py::arg("path"), py::arg("heartbeat"),
             py::arg("loop_tid"), py::arg("late_ms") = 10.0, py::arg("period_us") = 2000, py::arg("pid") = 0)
        .def("stop", &StallProbe::stop, py::call_guard<py::gil_scoped_release>())
        .def("samples", &StallProbe::samples);
}

}  // namespace upow

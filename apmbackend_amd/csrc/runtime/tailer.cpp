// Native log tailer: the MI355X-native replacement of perl_tail.pl + File::Tail
// (perl_tail.pl:13-42, stream_parse_transactions.js:902-975).
//
//  * one Tailer follows many files, reading whole-line chunks with pread() into one contiguous
//    batch buffer (ready for a single H2D copy), never splitting a line;
//  * the pause-file contract is kept: while `pause_file` exists nothing is read and the file
//    positions are held (perl_tail.pl:36-41);
//  * rotation / truncation is detected by inode change or a size smaller than the offset, and
//    the file is re-read from the start (File::Tail resetafter semantics, without the NFS inode
//    assertion the reference had to patch out);
//  * offsets persist across restarts (`save_offsets` / `load_offsets`), which the reference
//    lacked (restart = data gap).
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace py = pybind11;

namespace apm {

struct TailFile {
  std::string path;
  int32_t file_id;
  uint64_t offset = 0;
  uint64_t inode = 0;
  bool start_at_end = true;
};

class Tailer {
 public:
  Tailer(std::string pause_file, uint64_t max_batch_bytes)
      : pause_file_(std::move(pause_file)), max_batch_(max_batch_bytes) {}

  void add(const std::string& path, int32_t file_id, bool from_start) {
    TailFile f;
    f.path = path;
    f.file_id = file_id;
    f.start_at_end = !from_start;
    struct stat st;
    if (::stat(path.c_str(), &st) == 0) {
      f.inode = st.st_ino;
      f.offset = from_start ? 0 : (uint64_t)st.st_size;
    }
    files_.push_back(f);
  }

  bool paused() const {
    struct stat st;
    return !pause_file_.empty() && ::stat(pause_file_.c_str(), &st) == 0;
  }

  // Reads up to max_batch bytes of new complete lines. Returns (bytes, [(file_id, begin, end)]).
  std::pair<py::bytes, std::vector<std::tuple<int32_t, uint64_t, uint64_t>>> poll() {
    std::vector<std::tuple<int32_t, uint64_t, uint64_t>> chunks;
    std::string buf;
    if (paused()) return {py::bytes(buf), chunks};
    const size_t per_file = files_.empty() ? 0 : std::max<uint64_t>(65536, max_batch_ / files_.size());
    for (auto& f : files_) {
      if (buf.size() >= max_batch_) break;
      struct stat st;
      if (::stat(f.path.c_str(), &st) != 0) continue;
      if ((f.inode && (uint64_t)st.st_ino != f.inode) || (uint64_t)st.st_size < f.offset) {
        f.offset = 0;  // rotated or truncated
        f.inode = st.st_ino;
      }
      if (!f.inode) f.inode = st.st_ino;
      if ((uint64_t)st.st_size <= f.offset) continue;
      const uint64_t want = std::min<uint64_t>((uint64_t)st.st_size - f.offset, std::min<uint64_t>(per_file, max_batch_ - buf.size()));
      int fd = ::open(f.path.c_str(), O_RDONLY);
      if (fd < 0) continue;
      const size_t base = buf.size();
      buf.resize(base + want);
      ssize_t got = ::pread(fd, &buf[base], want, (off_t)f.offset);
      ::close(fd);
      if (got <= 0) { buf.resize(base); continue; }
      // cut at the last newline: partial lines stay in the file for the next poll
      size_t end = base + (size_t)got;
      while (end > base && buf[end - 1] != '\n') --end;
      buf.resize(end);
      if (end == base) continue;
      f.offset += end - base;
      chunks.emplace_back(f.file_id, (uint64_t)base, (uint64_t)end);
    }
    bytes_read_ += buf.size();
    return {py::bytes(buf), chunks};
  }

  void save_offsets(const std::string& path) const {
    std::string tmp = path + ".tmp";
    {
      std::ofstream o(tmp);
      o << "{";
      for (size_t i = 0; i < files_.size(); ++i) {
        if (i) o << ",";
        o << "\"" << files_[i].path << "\":[" << files_[i].offset << "," << files_[i].inode << "]";
      }
      o << "}";
      o.flush();
    }
    std::rename(tmp.c_str(), path.c_str());
  }

  void set_offset(const std::string& path, uint64_t offset, uint64_t inode) {
    for (auto& f : files_)
      if (f.path == path) { f.offset = offset; f.inode = inode; }
  }

  std::vector<std::tuple<std::string, uint64_t, uint64_t>> offsets() const {
    std::vector<std::tuple<std::string, uint64_t, uint64_t>> r;
    for (auto& f : files_) r.emplace_back(f.path, f.offset, f.inode);
    return r;
  }

  uint64_t bytes_read() const { return bytes_read_; }

 private:
  std::string pause_file_;
  uint64_t max_batch_;
  std::vector<TailFile> files_;
  uint64_t bytes_read_ = 0;
};

}  // namespace apm

void register_tailer(py::module_& m) {
  using apm::Tailer;
  py::class_<Tailer>(m, "Tailer")
      .def(py::init<std::string, uint64_t>(), py::arg("pause_file"), py::arg("max_batch_bytes") = 32ull << 20)
      .def("add", &Tailer::add, py::arg("path"), py::arg("file_id"), py::arg("from_start") = false)
      .def("poll", &Tailer::poll)
      .def("paused", &Tailer::paused)
      .def("save_offsets", &Tailer::save_offsets)
      .def("set_offset", &Tailer::set_offset)
      .def("offsets", &Tailer::offsets)
      .def("bytes_read", &Tailer::bytes_read);
}

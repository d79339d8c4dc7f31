#include "log_segment.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <map>

#include "common.h"
#include "json_host.h"

namespace dr {
namespace {

bool all_digits(const std::string& s, size_t b, size_t e) {
  if (b >= e) return false;
  for (size_t i = b; i < e; ++i) if (s[i] < '0' || s[i] > '9') return false;
  return true;
}

std::vector<std::string> split_dots(const std::string& s) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    size_t e = s.find('.', b);
    out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) return out;
    b = e + 1;
  }
}

struct Inst {  // CheckpointInstance (D/Checkpoints.scala:60-106)
  int64_t version;
  int parts;  // 0 = None (singular)
  bool operator<(const Inst& o) const {
    if (version != o.version) return version < o.version;
    return (parts ? parts : 1) < (o.parts ? o.parts : 1);
  }
  bool operator==(const Inst& o) const { return version == o.version && parts == o.parts; }
};

// getLatestCompleteCheckpointFromList (D/Checkpoints.scala:210-218)
bool latest_complete(const std::vector<Inst>& insts, int64_t not_later_than, Inst* out) {
  std::map<std::pair<int64_t, int>, int> groups;
  for (const Inst& i : insts)
    if (not_later_than < 0 || i.version <= not_later_than) groups[{i.version, i.parts}]++;
  bool found = false;
  for (auto& kv : groups) {
    Inst i{kv.first.first, kv.first.second};
    bool complete = i.parts == 0 ? kv.second == 1 : kv.second == i.parts;
    if (complete && (!found || *out < i)) { *out = i; found = true; }
  }
  return found;
}

// Checkpoints.lastCheckpoint (D/Checkpoints.scala:148-175): the first line of _last_checkpoint read
// as a CheckpointMetaData (Jackson: unknown fields ignored, an absent version reads as 0). A file
// that does not parse is "corrupted": the reference then lists the log for the latest complete
// checkpoint (findLastCompleteCheckpoint(MaxValue)), which is what listing from version 0 does here.
bool parse_last_checkpoint(const std::string& log_path, int64_t* version) {
  std::string p = log_path + "/_last_checkpoint";
  struct stat st;
  if (stat(p.c_str(), &st) != 0) return false;
  std::vector<uint8_t> b = read_file(p);
  size_t e = 0;
  while (e < b.size() && b[e] != '\n') ++e;
  JVal v;
  if (!json_parse(reinterpret_cast<const char*>(b.data()), e, &v) || v.t != JVal::OBJ) return false;
  const JVal* x = v.get("version");
  if (!x || x->t == JVal::NUL) { *version = 0; return true; }
  if (!x->is_int()) return false;
  *version = x->as_int();
  return true;
}

std::vector<std::string> list_dir(const std::string& path) {
  DIR* d = opendir(path.c_str());
  if (!d) fail(DR_E_EMPTY_DIR, fmt("No file found in the directory: %s.", path.c_str()));
  std::vector<std::string> names;
  while (dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n != "." && n != "..") names.push_back(n);
  }
  closedir(d);
  std::sort(names.begin(), names.end());
  return names;
}

uint64_t file_size(const std::string& path) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return 0;
  return uint64_t(st.st_size);
}

void verify_delta_versions(const std::vector<int64_t>& v) {  // D/SnapshotManagement.scala:365-372
  for (size_t i = 1; i < v.size(); ++i) {
    if (v[i] != v[0] + int64_t(i)) {
      std::string s;
      for (size_t j = 0; j < v.size(); ++j) { if (j) s += ", "; s += std::to_string(v[j]); }
      fail(DR_E_NONCONTIGUOUS, "Versions (Vector(" + s + ")) are not contiguous.");
    }
  }
}

LogSegmentInfo segment_from(const std::string& log_path, int64_t start_ckpt, int64_t version_to_load) {
  std::vector<std::string> names = list_dir(log_path);
  const int64_t start = start_ckpt < 0 ? 0 : start_ckpt;
  std::vector<std::string> files;
  for (const std::string& n : names) {
    bool ck = is_checkpoint_file(n), js = is_delta_file(n);
    if (!ck && !js) continue;
    int64_t v = file_version(n);
    if (v < start) continue;
    if (ck && file_size(log_path + "/" + n) == 0) continue;  // not atomically visible
    if (version_to_load >= 0 && v > version_to_load) break;
    files.push_back(n);
  }
  if (files.empty() && start_ckpt < 0)
    fail(DR_E_EMPTY_DIR, fmt("No file found in the directory: %s.", log_path.c_str()));
  if (files.empty()) return segment_from(log_path, -1, version_to_load);
  std::vector<std::string> cks, deltas;
  for (auto& n : files) (is_checkpoint_file(n) ? cks : deltas).push_back(n);
  std::vector<Inst> insts;
  for (auto& n : cks) insts.push_back({file_version(n), checkpoint_num_parts(n)});
  LogSegmentInfo seg;
  Inst nc{};
  if (latest_complete(insts, version_to_load, &nc)) {
    std::vector<int64_t> vers;
    for (auto& n : deltas) {
      int64_t v = file_version(n);
      if (v > nc.version) {
        seg.deltas.push_back({n, v, DR_FILE_JSON, 0});
        vers.push_back(v);
      }
    }
    if (!vers.empty()) {
      verify_delta_versions(vers);
      if (vers.front() != nc.version + 1)
        fail(DR_E_BAD_SEGMENT, fmt("requirement failed: Did not get the first delta file version: "
                                   "%lld to compute Snapshot", (long long)(nc.version + 1)));
      if (version_to_load >= 0 && vers.back() != version_to_load)
        fail(DR_E_BAD_SEGMENT, fmt("requirement failed: Did not get the last delta file version: "
                                   "%lld to compute Snapshot", (long long)version_to_load));
    }
    seg.version = vers.empty() ? nc.version : vers.back();
    seg.checkpoint_version = nc.version;
    for (auto& n : cks) {
      if (file_version(n) == nc.version && checkpoint_num_parts(n) == nc.parts)
        seg.checkpoint.push_back({n, nc.version, DR_FILE_CHECKPOINT, checkpoint_part(n)});
    }
    std::sort(seg.checkpoint.begin(), seg.checkpoint.end(),
              [](const SegFile& a, const SegFile& b) { return a.part < b.part; });
    return seg;
  }
  if (start_ckpt >= 0)
    fail(DR_E_MISSING_PART, fmt("Couldn't find all part files of the checkpoint version: %lld",  // D/DeltaErrors.scala:543-546
                                (long long)start_ckpt));
  std::vector<int64_t> vers;
  for (auto& n : deltas) {
    vers.push_back(file_version(n));
    seg.deltas.push_back({n, file_version(n), DR_FILE_JSON, 0});
  }
  verify_delta_versions(vers);
  if (vers.empty() || vers.front() != 0)
    // DeltaErrors.logFileNotFoundException (D/DeltaErrors.scala:451-457). The listing has no
    // metadata, so the text carries the default delta.logRetentionDuration /
    // delta.checkpointRetentionDuration (D/DeltaConfig.scala:251-281) as Spark's
    // CalendarInterval.toString renders them -- the reference's text on a first load; a host that
    // holds a snapshot's metadata re-renders the configured values (delta_amd/delta_log.py:
    // retention_text, used by DeltaLog.update)
    fail(DR_E_LOG_TRUNCATED, fmt("%s/%020lld.json: Unable to reconstruct state at version %lld as the "
                                 "transaction log has been truncated due to manual deletion or the log "
                                 "retention policy (delta.logRetentionDuration=30 days) and checkpoint "
                                 "retention policy (delta.checkpointRetentionDuration=2 days)",
                                 log_path.c_str(), 0LL, (long long)(vers.empty() ? -1 : vers.back())));
  if (version_to_load >= 0 && vers.back() != version_to_load)
    fail(DR_E_BAD_SEGMENT, fmt("requirement failed: Did not get the last delta file version: "
                               "%lld to compute Snapshot", (long long)version_to_load));
  seg.version = vers.back();
  return seg;
}

}  // namespace

bool is_delta_file(const std::string& n) {  // \d+\.json
  size_t d = n.size() >= 5 ? n.size() - 5 : 0;
  return n.size() > 5 && n.compare(d, 5, ".json") == 0 && all_digits(n, 0, d);
}

bool is_checkpoint_file(const std::string& n) {  // \d+\.checkpoint(\.\d+\.\d+)?\.parquet
  auto s = split_dots(n);
  if (s.size() == 3) return all_digits(s[0], 0, s[0].size()) && s[1] == "checkpoint" && s[2] == "parquet";
  if (s.size() == 5)
    return all_digits(s[0], 0, s[0].size()) && s[1] == "checkpoint" && all_digits(s[2], 0, s[2].size()) &&
           all_digits(s[3], 0, s[3].size()) && s[4] == "parquet";
  return false;
}

int64_t file_version(const std::string& n) { return std::stoll(n.substr(0, n.find('.'))); }

int checkpoint_num_parts(const std::string& n) {
  auto s = split_dots(n);
  return s.size() == 5 ? std::stoi(s[3]) : 0;
}

int checkpoint_part(const std::string& n) {
  auto s = split_dots(n);
  return s.size() == 5 ? std::stoi(s[2]) : 0;
}

LogSegmentInfo get_log_segment(const std::string& log_path, int64_t version_to_load) {
  int64_t lc = -1;
  if (!parse_last_checkpoint(log_path, &lc)) lc = -1;
  if (version_to_load >= 0 && lc > version_to_load) lc = -1;
  struct stat st;
  if (stat(log_path.c_str(), &st) != 0)
    fail(DR_E_EMPTY_DIR, fmt("No file found in the directory: %s.", log_path.c_str()));
  return segment_from(log_path, lc, version_to_load);
}

std::vector<uint8_t> read_file(const std::string& path) {
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) fail(DR_E_IO, fmt("cannot open %s", path.c_str()));
  struct stat st;
  fstat(fd, &st);
  std::vector<uint8_t> b(size_t(st.st_size));
  size_t got = 0;
  while (got < b.size()) {
    ssize_t r = read(fd, b.data() + got, b.size() - got);
    if (r <= 0) { close(fd); fail(DR_E_IO, fmt("read failed on %s", path.c_str())); }
    got += size_t(r);
  }
  close(fd);
  return b;
}



uint64_t file_size(const std::string& path) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) fail(DR_E_IO, fmt("cannot stat %s", path.c_str()));
  return uint64_t(st.st_size);
}

std::vector<uint8_t> read_tail(const std::string& path, uint64_t n) {
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) fail(DR_E_IO, fmt("cannot open %s", path.c_str()));
  struct stat st;
  fstat(fd, &st);
  const uint64_t sz = uint64_t(st.st_size);
  const uint64_t k = std::min<uint64_t>(n, sz);
  std::vector<uint8_t> b(static_cast<size_t>(k));
  size_t got = 0;
  while (got < b.size()) {
    ssize_t r = pread(fd, b.data() + got, b.size() - got, off_t(sz - k + got));
    if (r <= 0) { close(fd); fail(DR_E_IO, fmt("read failed on %s", path.c_str())); }
    got += size_t(r);
  }
  close(fd);
  return b;
}

}  // namespace dr

// LogSegment construction from a _delta_log listing (POSIX), restating
// SnapshotManagement.getLogSegmentForVersion / verifyDeltaVersions
// (D/SnapshotManagement.scala:82-179,365-372), Checkpoints.lastCheckpoint and
// getLatestCompleteCheckpointFromList (D/Checkpoints.scala:148-218) and FileNames
// (D/util/FileNames.scala:25-107).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dr {

struct SegFile {
  std::string name;     // file name inside the log directory
  int64_t version;
  int kind;             // DR_FILE_JSON / DR_FILE_CHECKPOINT
  int part;             // 1-based part index for multi-part checkpoints, 0 otherwise
};

struct LogSegmentInfo {
  int64_t version = -1;
  int64_t checkpoint_version = -1;   // -1: none
  std::vector<SegFile> checkpoint;   // parts in part order
  std::vector<SegFile> deltas;       // ascending versions
};

bool is_delta_file(const std::string& name);
bool is_checkpoint_file(const std::string& name);
int64_t file_version(const std::string& name);
int checkpoint_num_parts(const std::string& name);   // 0 = singular
int checkpoint_part(const std::string& name);        // 0 = singular

// version_to_load < 0: latest.
LogSegmentInfo get_log_segment(const std::string& log_path, int64_t version_to_load);

std::vector<uint8_t> read_file(const std::string& path);
uint64_t file_size(const std::string& path);
// The last `n` bytes of a file (all of it when shorter).
std::vector<uint8_t> read_tail(const std::string& path, uint64_t n);

}  // namespace dr

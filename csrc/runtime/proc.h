// Process liveness on this node, shared by the step channel and the vote board.
#pragma once
#include <errno.h>
#include <signal.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

namespace pk {

// A process runs (same node: every rank of a group shares the host).  EPERM means it exists but
// belongs to another user.  A killed process that its parent has not reaped yet (a zombie)
// still answers kill(pid, 0): its /proc state decides (a rank must not wait on a dead peer just
// because nobody called wait() on it).
inline bool pid_alive(int32_t pid) {
  if (pid <= 0) return true;
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[48];
  std::snprintf(path, sizeof path, "/proc/%d/stat", static_cast<int>(pid));
  FILE* f = std::fopen(path, "r");
  if (f == nullptr) return errno != ENOENT;
  char buf[512];
  const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');  // "pid (comm) S ...": comm may hold spaces / parens
  return !(rp != nullptr && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}

}  // namespace pk

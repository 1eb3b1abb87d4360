// Re-shard merge of engine checkpoints (elastic degrade / grow).
//
// The reference restarts each stage from its resume file with every per-series history intact
// (stream_calc_stats.js:54-87, stream_calc_z_score.js:37-64, stream_process_alerts.js:111-142).
// When the supervisor restarts a rank group at another world size, the JVM hosts are sharded
// anew and a new rank owns servers that several old ranks held.  merge_checkpoints() builds that
// rank's starting state from the old ranks' checkpoints, on the host (no GPU), as one ordinary
// checkpoint file that Engine::load_state reads:
//   * per series (window buckets + spill samples, z-score rings / moments / lengths, alert
//     counters, NaN horizons, settings), per server (emission rank, node-wide index), per file
//     (SOAP context, open audit block, parse carry), per raw service (registry), the GPU join's
//     key table, need arena and chain blocks, and the pending release lines -- the parts whose
//     server the new rank owns, renumbered into its own ids;
//   * node-wide state (clocks, bucket slots, alert cooldowns) from the inputs, which agree: the
//     inputs are the old ranks' states at one common batch (lock-step ranks checkpoint at the
//     same batches; each chain file is a complete small state, so any chain prefix is one).
// The join's table keys mix in world-invariant server / file keys (devjoin_dev.h gkey_of,
// aud_key), so they stay valid under the new numbering.  A carried audit-trail map entry has no
// file field: an input's entries are all kept (entries of files this rank does not own are never
// matched and stay inert).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace apm {

struct MergeResult {
  uint64_t batch_no = 0;        // the common batch the inputs were taken at
  int64_t series = 0, keys = 0, need = 0, pending = 0, raw = 0, files = 0, servers = 0;
  std::vector<std::string> used;  // the checkpoint file of each input that was merged
  std::vector<std::string> extras;  // their SEC_EXTRA payloads (tail offsets ...), input order
};

// Batch numbers of the files of a checkpoint (a chain manifest or one file), in chain order.
std::vector<std::pair<uint64_t, std::string>> checkpoint_batches(const std::string& path);

// inputs: each old rank's checkpoint (`<prefix>.ckpt` chain manifest, or a single file).
// keep_servers: the servers the new rank owns.  batch_no: the batch to merge at (0: the newest
// batch present in every input).  Writes `out_path` (atomic) with `extra` as its SEC_EXTRA.
MergeResult merge_checkpoints(const std::vector<std::string>& inputs, const std::vector<std::string>& keep_servers,
                              const std::string& out_path, const std::string& extra, uint64_t batch_no = 0);

}  // namespace apm

/*
 * trivy_secret.h -- C ABI of the MI355X secret-scan engine (libtrivy_secret.so).
 *
 * Drop-in boundary for trivy's secret hot path, pkg/fanal/secret:
 *
 *   reference (Go)                                    this ABI
 *   ------------------------------------------------  ---------------------------------
 *   secret.NewScanner(*Config) Scanner                tsg_ruleset_compile
 *       scanner.go:293-329 (rule assembly stays in the host language; the final
 *       Global{Rules, AllowRules, ExcludeBlock} is handed over here)
 *   regexp compile error via Regexp.UnmarshalYAML     TSG_ERR_CONFIG + err text
 *       scanner.go:69-81
 *   Global.AllowPath(path) bool                       tsg_ruleset_allow_path
 *       scanner.go:55-57 (used by SecretAnalyzer.Required, analyzer/secret/secret.go:145)
 *   (*Scanner).Scan(ScanArgs) types.Secret            tsg_scan_cpu (one file, exact CPU)
 *       scanner.go:341-416                            tsg_scan_batch (many files, GPU)
 *   SecretAnalyzer.Analyze per-file goroutines        tsg_queue_scan (concurrent callers
 *       analyzer/secret/secret.go:78-110,               coalesced into pinned batches),
 *       analyzer.go:419-443                             tsg_slot_* / tsg_scan_batch (batches)
 *   per-layer goroutines over a node's GPUs           tsg_multi_* (one process, N devices)
 *       artifact/image/image.go:210-234
 *
 * Error convention: every call returns TSG_OK (0) or a negative TSG_ERR_*; the
 * message of the last failing call on this thread is tsg_last_error().  No C++
 * exception crosses the ABI.  Every entry point is thread-safe (the GPU calls name the
 * caller's own slot and submission ticket; none acts on "the last" batch); a tsg_ruleset
 * is immutable and may be shared by any number of threads and contexts.  The library never
 * retains a caller pointer past a call.
 *
 * Result format (tsg_result_data), little endian:
 *   u32 magic 'TSG1' (0x31475354), u32 nfiles, then per file:
 *     u8  status      0 = no findings  -> types.Secret{}             (scanner.go:401-403)
 *                     1 = path allowed -> types.Secret{FilePath}      (scanner.go:343-347)
 *                     2 = findings     -> types.Secret{FilePath, Findings}
 *     u32 nfindings, then per finding (already in Go sort.Slice order, scanner.go:405-410):
 *       u32 rule (index into the compiled rule list: RuleID/Category/Severity/Title)
 *       i32 start_line, i32 end_line, bytes match, u32 nlines, then per line:
 *         i32 number, u8 flags (1 IsCause, 2 FirstCause, 4 LastCause), bytes content
 *   bytes = u32 length + raw bytes (Content == Highlighted in the reference).
 */
#ifndef TRIVY_SECRET_H
#define TRIVY_SECRET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSG_OK 0
#define TSG_ERR_CONFIG -1  /* a regex failed to compile (Go regexp syntax) */
#define TSG_ERR_ARG -2     /* bad argument */
#define TSG_ERR_GPU -3     /* HIP runtime / device failure */
#define TSG_ERR_NOMEM -4   /* allocation failure */
#define TSG_ERR_INTERNAL -5

/* secret.AllowRule (scanner.go:186-191). NULL regex/path = field absent. */
typedef struct tsg_allow_rule_desc {
  const char* id;
  const char* description;
  const char* regex;
  const char* path;
} tsg_allow_rule_desc;

/* secret.Rule (scanner.go:83-94). NULL regex/path = field absent. */
typedef struct tsg_rule_desc {
  const char* id;
  const char* category;
  const char* title;
  const char* severity;
  const char* regex;
  const char* const* keywords;
  uint32_t n_keywords;
  const char* path;
  const tsg_allow_rule_desc* allow_rules;
  uint32_t n_allow_rules;
  const char* const* exclude_regexes; /* ExcludeBlock.Regexes */
  uint32_t n_exclude_regexes;
  const char* secret_group_name;
} tsg_rule_desc;

typedef struct tsg_ruleset tsg_ruleset;
typedef struct tsg_result tsg_result;
typedef struct tsg_ctx tsg_ctx;

/* Compile Global{Rules, AllowRules, ExcludeBlock}: regexes, the K1 keyword automaton,
 * the K2 rule-group DFAs.  On TSG_ERR_CONFIG, err holds Go's error text. */
int tsg_ruleset_compile(const tsg_rule_desc* rules, uint32_t n_rules,
                        const tsg_allow_rule_desc* allow_rules, uint32_t n_allow_rules,
                        const char* const* exclude_regexes, uint32_t n_exclude_regexes,
                        tsg_ruleset** out, char* err, size_t err_len);
void tsg_ruleset_destroy(tsg_ruleset* rs);

/* Global.AllowPath: 1 allowed, 0 not, <0 error. */
int tsg_ruleset_allow_path(const tsg_ruleset* rs, const char* path, size_t path_len);

typedef struct tsg_ruleset_info {
  uint32_t n_rules;
  uint32_t n_keywords;      /* K1 keyword ids incl. 3 fallback pseudo keywords */
  uint32_t n_groups;        /* K2 DFAs */
  uint32_t n_hostonly;      /* rules without a GPU DFA (state cap) */
  uint32_t kw_states;       /* K1 automaton states */
  uint32_t max_group_states;
  uint64_t table_bytes;     /* all device tables */
  uint32_t kw_classes;      /* K1 automaton byte classes */
  uint32_t k1x_literals;    /* literals of the hashed prefilter (K1X; large rule sets) */
} tsg_ruleset_info;
int tsg_ruleset_get_info(const tsg_ruleset* rs, tsg_ruleset_info* out);

/* Exact CPU Scan of one file (scanner.go:341-416). */
int tsg_scan_cpu(const tsg_ruleset* rs, const char* path, size_t path_len,
                 const uint8_t* content, size_t len, tsg_result** out);

/* Exact CPU Scan of a batch: file i = data[offsets[i] .. offsets[i+1]),
 * path i = paths[path_offsets[i] .. path_offsets[i+1]). nthreads <= 0: hardware. */
int tsg_scan_cpu_batch(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                       uint32_t nfiles, const char* paths, const uint64_t* path_offsets,
                       int nthreads, tsg_result** out);

const uint8_t* tsg_result_data(const tsg_result* r, size_t* len);

/* sort.Slice with Go 1.19's pdqsort_func (unstable; ties ordered exactly as Go orders them)
 * of n items by (key bytes as a Go string, then secondary if not NULL): perm[k] = index of
 * the k-th item.  Replaces the secret part of AnalysisResult.Sort
 * (pkg/fanal/analyzer/analyzer.go:212-223): files by FilePath, findings by (RuleID,
 * StartLine). */
int tsg_go_sort_perm(const uint8_t* keys, const uint64_t* key_offsets, const int64_t* secondary,
                     uint32_t n, uint32_t* perm);
void tsg_result_free(tsg_result* r);
/* Counts of a result (bench and test checks): files, files with findings, findings. */
int tsg_result_summary(const tsg_result* r, uint64_t* nfiles, uint64_t* files_with_findings,
                       uint64_t* findings);

/* ---- GPU (one context per device) ----
 *
 * A context owns the rule tables on one device, two lanes (HIP stream + HBM buffers: the
 * H2D of one batch overlaps the kernels of the other), a pool of pinned host slots that
 * batches are staged in, and the host resolvers of batches in flight.  The library never
 * retains a caller pointer past a call (batch bytes are copied into, or written directly
 * by the caller into, library-owned pinned slots).
 *
 * Threading: every entry point below is thread-safe on a shared context.  No call acts on
 * "the last" anything: a caller names its own slot (slot id) and its own submission
 * (ticket), so concurrent per-layer / per-file callers (image.go:210-234,
 * analyzer.go:419-443) never see each other's batches. */
typedef struct tsg_ctx_options {
  uint32_t chunk_bytes;      /* bytes per lane (multiple of 16); 0 = default */
  uint32_t ext_cap;          /* max bytes a lane follows a match past its chunk; 0 = default */
  uint32_t cand_capacity;    /* candidate records per batch; 0 = default */
  int32_t host_threads;      /* resolver threads; <= 0 = 16 */
  uint32_t adapt_mib;        /* first batch of at least this many MiB samples K1's literal
                                frequencies and stops reporting the frequent ones (their
                                keyword gates are then checked on the host); 0 = 16,
                                0xFFFFFFFF = never */
  uint32_t flags;            /* TSG_CTX_* */
  uint32_t slot_mib;         /* default capacity of a pinned slot (tsg_queue batches,
                                tsg_multi pieces); 0 = 256 */
  uint32_t max_slots;        /* pinned slots a context may hold; 0 = 16 */
} tsg_ctx_options;

/* Test mode: no HIP device is touched; the kernels' algorithm is emulated on the CPU over
 * the same slots, lanes and queue logic (tests of the pipeline and of tsg_queue on hosts
 * without a GPU).  Never chosen implicitly. */
#define TSG_CTX_EMULATE 1u

int tsg_ctx_create(int device, const tsg_ruleset* rs, const tsg_ctx_options* opt,
                   tsg_ctx** out);
/* Waits for every batch in flight, then frees the context. */
void tsg_ctx_destroy(tsg_ctx* ctx);

/* -- Zero-copy staging: the caller packs files straight into a pinned slot -------------
 * Replaces the per-file io.ReadAll copy of SecretAnalyzer.Analyze
 * (pkg/fanal/analyzer/secret/secret.go:85): ingest writes file bytes into the slot;
 * offsets[0] = path_offsets[0] = 0 and file i = data[offsets[i] .. offsets[i+1]),
 * path i = paths[path_offsets[i] .. path_offsets[i+1]). */
typedef struct tsg_slot_view {
  uint32_t id;
  uint8_t* data;            /* data_cap bytes */
  uint64_t data_cap;
  uint64_t* offsets;        /* files_cap + 1 */
  uint32_t files_cap;
  char* paths;              /* paths_cap bytes */
  uint64_t paths_cap;
  uint64_t* path_offsets;   /* files_cap + 1 */
} tsg_slot_view;
/* A free slot with at least these capacities (allocated or grown if needed), owned by the
 * caller until tsg_slot_release.  Waits while every slot is busy with submissions. */
int tsg_slot_acquire(tsg_ctx* ctx, uint64_t data_bytes, uint32_t nfiles, uint64_t path_bytes,
                     tsg_slot_view* out);
/* Submit the slot's first nfiles files: the device part runs asynchronously, the host
 * resolution follows it on the resolver pool.  *ticket names this submission for
 * tsg_batch_collect.  The slot may be submitted again (same bytes) at once, also with a
 * different nfiles: a submission reads the slot and never writes the bytes the caller can
 * reach (only a slot the library filled itself -- tsg_batch_upload -- submitted whole and
 * with nothing else in flight carries its zero tail and offsets in the room behind data_cap).
 * The slot must not be written until its submissions are collected. */
int tsg_slot_submit(tsg_ctx* ctx, uint32_t slot_id, uint32_t nfiles, uint64_t* ticket);
/* Give the slot back to the context (it is reused once its submissions are done). */
int tsg_slot_release(tsg_ctx* ctx, uint32_t slot_id);

/* -- Copying staging: the batch is copied into a free slot, which is then the caller's
 * (submit it with tsg_slot_submit, give it back with tsg_slot_release). */
int tsg_batch_upload(tsg_ctx* ctx, const uint8_t* data, const uint64_t* offsets,
                     uint32_t nfiles, const char* paths, const uint64_t* path_offsets,
                     uint32_t* slot_id);
/* Results of one submission (waits for its resolution); each ticket is collected once. */
int tsg_batch_collect(tsg_ctx* ctx, uint64_t ticket, tsg_result** out);
/* number of submitted, uncollected tickets of the context (all callers) */
int tsg_batch_pending(const tsg_ctx* ctx);
/* One batch, synchronously: copied into a slot of its own, scanned, resolved, slot freed
 * (the Scan of many files; thread-safe, any number of concurrent callers). */
int tsg_scan_batch(tsg_ctx* ctx, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                   const char* paths, const uint64_t* path_offsets, tsg_result** out);
/* Test hook: the device part of a scan of an acquired slot's first nfiles files,
 * synchronously, without resolution; writes K1's keyword bits [nfiles * kw_words] and chunk
 * event bits [ceil(bytes / chunk_bytes)] (either pointer may be NULL). */
int tsg_batch_kernels(tsg_ctx* ctx, uint32_t slot_id, uint32_t nfiles, uint32_t* kw,
                      size_t kw_len, uint32_t* ev, size_t ev_len);

typedef struct tsg_stats {
  double k1_ms;          /* K1 literal automaton + run counters, last collected batch (HIP events) */
  double k2_ms;          /* K2 rule-group DFAs (the persistent work-list launch) */
  double aux_ms;         /* the outputs kernel (results into pinned, host-mapped memory) */
  double resolve_ms;     /* host exact resolution (wall) */
  uint64_t bytes;        /* content bytes of the batch */
  uint64_t k2_bytes;     /* chunk bytes K2 scans (items listed x chunk) */
  uint64_t candidates;   /* candidate records produced */
  uint64_t files_resolved;  /* files with findings */
  uint32_t k2_launches;  /* K2 work-list entries */
  uint32_t overflow;     /* 1 if the candidate buffer overflowed (files resolved whole) */
  double gate_ms;        /* keyword gates + items + device-side layout */
  uint64_t k2_items;     /* (file, chunk) items K2 scanned */
  uint32_t k1_hot_states;  /* K1 automaton states no longer reported (adaptation) */
  double h2d_ms;         /* H2D of the batch (pinned slot -> HBM) */
  uint32_t groups_skipped; /* rule groups K2 left to the host (item capacity) */
  uint64_t batches;      /* batches collected so far, and their sums: */
  uint64_t sum_bytes;
  double sum_k1_ms, sum_gate_ms, sum_k2_ms, sum_h2d_ms, sum_d2h_ms, sum_resolve_ms;
  double wait_ms;        /* last batch: its kernels waiting for the previous batch's */
  /* K2 diagnostics of the last batch (TSG_K2_DIAG=1 in the environment, else 0): bytes
   * followed past chunk ends, the longest such tail, tails over 4 KiB, words replayed for
   * accepts */
  uint32_t k2_tail_bytes, k2_tail_max, k2_long_tails, k2_replays;
  /* the rest of a batch's device work (HIP events on its lane): the prep kernel (zero fills,
   * coarse file map) and the H2D of the file offsets; aux_ms / sum_d2h_ms above are the
   * outputs kernel (results written into pinned, host-mapped memory) */
  double prep_ms, meta_ms, sum_prep_ms, sum_meta_ms;
  /* K1X (large rule sets) in the last batch: 16-B words listed with a prefilter hit, and
   * words verified inline because their block's list slice was full */
  uint32_t k1x_records, k1x_inline;
  /* K1F (the filter-and-verify K1) in the last batch: 16-B words listed with a filter hit,
   * and literal occurrences its verification confirmed */
  uint32_t k1f_listed, k1f_arrivals;
  /* chunks of the last batch whose K1 event word is not empty (the item passes' units) */
  uint32_t event_chunks;
  /* 1: K1 ran as the filter-and-verify K1F (k1f_kernel), 0: as the automaton (k1_kernel) */
  uint32_t k1_filter;
  /* last batch, by the device wall clock stamped inside the kernels (0 when K1 was not
   * K1F): K1F's first block start to its last block end; K1F's start to K2's last block
   * end (every kernel and gap of the chain); the gates pass's start to K2's end */
  double k1_clock_ms, chain_clock_ms, post_k1_clock_ms;
  /* their sums over the batches collected so far */
  double sum_k1_clock_ms, sum_chain_clock_ms, sum_post_k1_clock_ms;
} tsg_stats;
int tsg_ctx_get_stats(const tsg_ctx* ctx, tsg_stats* out);

/* -- Submission queue for concurrent per-file callers ----------------------------------
 * The analyzer framework calls Analyze -> Scan from one goroutine per file
 * (pkg/fanal/analyzer/analyzer.go:419-443).  tsg_queue_scan is that Scan: any number of
 * threads call it at once; their files are packed into the open slot, a slot is submitted
 * when full or flush_us after its first file, and each call returns its own file's result
 * (tsg_result, one file, the format above) once its batch is resolved.  Files too large
 * for a slot are scanned by the exact CPU path (same results). */
typedef struct tsg_queue tsg_queue;
int tsg_queue_create(tsg_ctx* ctx, uint32_t flush_us, tsg_queue** out);
int tsg_queue_scan(tsg_queue* q, const char* path, size_t path_len, const uint8_t* content,
                   size_t len, tsg_result** out);
/* submit the open slot now */
int tsg_queue_flush(tsg_queue* q);
/* waits for every call in flight */
void tsg_queue_destroy(tsg_queue* q);

/* -- One process, several GPUs (multi.cpp) ------------------------------------------
 * trivy is one process: per-layer goroutines (pkg/fanal/artifact/image/image.go:210-234)
 * and per-file goroutines (pkg/fanal/analyzer/analyzer.go:419-443) drive every GPU of the
 * node from one address space.  tsg_multi holds one context per device (same options);
 * tsg_multi_scan_batch shards a batch's files over them, largest first onto the least
 * loaded device (LPT by bytes), copies each share straight into that device's pinned
 * slots (pieces of slot_mib), and returns the results in input order (tsg_result format),
 * identical to tsg_scan_batch on one context.  Thread-safe; no collective. */
typedef struct tsg_multi tsg_multi;
int tsg_multi_create(const int* devices, uint32_t n, const tsg_ruleset* rs,
                     const tsg_ctx_options* opt, tsg_multi** out);
int tsg_multi_size(const tsg_multi* m);
/* the i-th device's context (owned by m; e.g. for a tsg_queue per device) */
int tsg_multi_ctx(tsg_multi* m, uint32_t i, tsg_ctx** out);
int tsg_multi_scan_batch(tsg_multi* m, const uint8_t* data, const uint64_t* offsets,
                         uint32_t nfiles, const char* paths, const uint64_t* path_offsets,
                         tsg_result** out);
int tsg_multi_get_stats(const tsg_multi* m, uint32_t i, tsg_stats* out);
void tsg_multi_destroy(tsg_multi* m);

const char* tsg_last_error(void);

/* ---- test and measurement knobs ----
 * Process-wide switches that change how (never what) the library computes, for tests and
 * measurements only.  They are set through this call alone: the library reads no
 * environment variable that changes a plan, a kernel or a result (the profiling switches
 * TSG_PROF, TSG_PROF2, TSG_LAYER_PROF, TSG_K2_DIAG, TSG_K2_TRACE, TSG_K1F_TRACE and TSG_DEBUG_RESOLVE only
 * add timings, counters or traces).  value NULL or "" resets the knob.
 *   "tar_range_kib"   sub-range floor of the parallel tar index walk (default 64 MiB)
 *   "piece_mib"       piece floor of tsg_layer_scan / tsg_fs_scan (default 16)
 *   "pike_only"       "1": the Go-regexp matcher uses the Pike VM alone (no backtracker)
 *   "no_k1x"          "1": a rule set too large for K1's automaton is not split onto K1X
 *   "x_step"          1, 2 or 4: the K1X window step of the next plans (default: the widest
 *                     step whose K1 automaton fits the packed table)
 *   "emu_wordrec"     "1": emulated K2 writes one record per accepting 16-B word, as the
 *                     kernel does (tsg_scan_batch_emulated, TSG_CTX_EMULATE contexts)
 *   "emu_kw_unknown"  comma-separated keywords the emulated K1 leaves to the host, as
 *                     after its adaptation (tsg_scan_batch_emulated)
 *   "k1_automaton"    "1": contexts created next run K1 as the LDS automaton instead of the
 *                     filter-and-verify K1F (k1f.hpp)
 *   "group_states"    state cap of a K2 rule-group DFA in the next compiled rule sets
 *                     (default 2,048 for rule sets of up to 256 rules, else 1,024)
 *   "group_table_kib" table cap of a K2 rule-group DFA, 1..64 KiB (default 64 for rule
 *                     sets of up to 256 rules, else 48)
 *   "k1f_grid"        cap on K1F's blocks (default: one per CU): many tiles per wave in
 *                     small test batches
 *   "k1f_list"        "1": K1F lists the chunks with events itself (no gates pass; the item
 *                     passes gate files from their keyword bits)
 * Returns TSG_ERR_ARG for an unknown name. */
int tsg_test_knob(const char* name, const char* value);

/* ---- test hooks: the Go-regexp engine and the DFA builder in isolation ---- */
typedef struct tsg_regex tsg_regex;
int tsg_regex_compile(const char* src, tsg_regex** out, char* err, size_t err_len);
void tsg_regex_free(tsg_regex* re);
int tsg_regex_num_slots(const tsg_regex* re);
/* regexp.MatchString: 1 / 0 */
int tsg_regex_match(const tsg_regex* re, const uint8_t* text, size_t len);
/* FindAllIndex (submatch=0, 2 slots/match) or FindAllSubmatchIndex (submatch=1).
 * Writes up to cap int64 values, returns the number of values needed (>= 0). */
int64_t tsg_regex_find_all(const tsg_regex* re, const uint8_t* text, size_t len, int submatch,
                           int64_t* out, size_t cap);
/* FindAll with a chosen matcher: 0 auto, 1 Pike VM only, 2 bit-state backtracker where
 * its visited table fits (results must not depend on the choice). */
int64_t tsg_regex_find_all_engine(const tsg_regex* re, const uint8_t* text, size_t len,
                                  int submatch, int engine, int64_t* out, size_t cap);
/* DFA candidate end offsets of one regex over text (all p where a match may end),
 * computed with the GPU lane algorithm (chunk bytes per lane). Returns count. */
int64_t tsg_regex_dfa_ends(const tsg_regex* re, const uint8_t* text, size_t len, uint32_t chunk,
                           int64_t* out, size_t cap);

/* Emulate K1+K2 on the CPU (no resolution) and report, per rule, the number of
 * candidate end offsets, and per rule group the bytes K2 scans (plan tuning). */
int tsg_emulate_candidate_stats(const tsg_ruleset* rs, const uint8_t* data,
                                const uint64_t* offsets, uint32_t nfiles, uint32_t chunk,
                                uint64_t* cand_per_rule, uint64_t* gated_bytes_per_group);

/* K1 reference semantics on the CPU (plan.hpp k1_reference): same layout as
 * tsg_batch_k1_output. */
int tsg_emulate_k1(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                   uint32_t nfiles, uint32_t chunk, uint32_t* kw, size_t kw_len, uint32_t* ev,
                   size_t ev_len);

/* K1F (the filter-and-verify K1, k1f.hpp) emulated on the CPU with the device's tables and
 * bit logic: keyword bits and chunk events in tsg_emulate_k1's layout; the literals listed
 * in quiet_ids are left out of the filter (the adaptation's hot literals), and with
 * sample_kib > 0 the filter is priced on the batch's first sample_kib KiB (as the
 * adaptation prices it on a sample of its batch).  stats (or NULL): {flagged word groups,
 * verified literal occurrences, records in the filter, 0}.  TSG_ERR_CONFIG when K1F does
 * not apply to the rule set (the automaton K1 runs then). */
int tsg_emulate_k1f(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                    uint32_t nfiles, uint32_t chunk, const uint32_t* quiet_ids, uint32_t nquiet,
                    uint32_t sample_kib, uint32_t* kw, size_t kw_len, uint32_t* ev, size_t ev_len,
                    uint64_t* stats);

/* Plan introspection: per rule group id (-1 host-only), relaxation (-1 exact), max len. */
int tsg_ruleset_rule_plan(const tsg_ruleset* rs, uint32_t rule, int32_t* group, int32_t* relax,
                          int64_t* max_len);

/* Plan introspection: the rule's K1 event bits (1 run U, 2 run D, 4.. literal classes,
 * 1<<31 none), the largest distance from a GPU-program match start to its event byte,
 * and a description of the anchor. */
int tsg_ruleset_rule_anchor(const tsg_ruleset* rs, uint32_t rule, uint32_t* event, int64_t* evdist,
                            char* desc, size_t desc_len);

/* Plan introspection: K1 literal i (0 <= i < n; ids below tsg_ruleset_info.n_keywords are
 * keywords, the rest anchor literals): its bytes (min(len, cap) copied), length and event
 * bits.  TSG_ERR_ARG once i >= n. */
int tsg_ruleset_k1_literal(const tsg_ruleset* rs, uint32_t i, uint8_t* buf, uint32_t cap,
                           uint32_t* len, uint32_t* event);

/* Emulate K1+K2 on the CPU with the GPU algorithm and resolve (tests). */
int tsg_scan_batch_emulated(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                            uint32_t nfiles, const char* paths, const uint64_t* path_offsets,
                            uint32_t chunk, tsg_result** out);

/* Layer ingest, replaces walker.LayerTar.Walk (pkg/fanal/walker/tar.go:33-84)
 * + AnalyzerGroup.AnalyzeFile's Required gate (analyzer.go:399-409) + SecretAnalyzer.Required
 * (analyzer/secret/secret.go:112-150) + utils.IsBinary (utils.go:71-89): walks an uncompressed
 * layer tar held in memory and packs every file the secret analyzer would scan into one batch
 * (paths get the "/" prefix of image files, secret.go:90-96).  skip_files / skip_dirs are the
 * walker's --skip-files / --skip-dirs; config_path the secret config (Required skips its base
 * name).  A malformed archive is TSG_ERR_ARG ("failed to extract the archive", tar.go:40). */
typedef struct tsg_layer tsg_layer;
typedef struct tsg_layer_view {
  const uint8_t* data;           /* kept files back to back (tsg_batch_upload layout) */
  const uint64_t* offsets;       /* [nfiles + 1] */
  uint32_t nfiles;
  const uint8_t* paths;          /* scan paths back to back */
  const uint64_t* path_offsets;  /* [nfiles + 1] */
  const char* opq;               /* opaque dirs, each NUL-terminated (tar.go:48-51) */
  size_t opq_len;
  const char* wh;                /* whiteout files, each NUL-terminated (tar.go:53-57) */
  size_t wh_len;
  uint32_t walked;               /* regular files the walker handed to the analyzers */
} tsg_layer_view;
int tsg_layer_pack(const tsg_ruleset* rs, const uint8_t* tar, uint64_t tar_len,
                   const char* const* skip_files, uint32_t n_skip_files,
                   const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                   tsg_layer** out);
/* Rank `rank` of `world`'s share of the same layer (configs[2], one layer sharded across the
 * GPUs of a node): the header chain, whiteouts, opaque dirs and skip-dir logic are those of
 * the whole layer (every rank returns the same opq / wh / walked); the walked regular files
 * are cut into `world` contiguous runs of about equal bytes in archive order, and only this
 * rank's run is gated and packed.  The union over ranks equals tsg_layer_pack's batch. */
int tsg_layer_pack_shard(const tsg_ruleset* rs, const uint8_t* tar, uint64_t tar_len,
                         const char* const* skip_files, uint32_t n_skip_files,
                         const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                         uint32_t rank, uint32_t world, tsg_layer** out);
int tsg_layer_get(const tsg_layer* layer, tsg_layer_view* out);
/* The header index itself split over the ranks (configs[2] at N GPUs; replaces the whole-chain
 * walk of tar.go:33-84 that tsg_layer_pack_shard repeats on every rank).  Rank r owns the
 * entries whose header group starts in its 512-aligned byte range [lo, hi) of the tar.
 *   1. tsg_layer_range_walk: speculative walk of the range from its first block that
 *      checksums as a ustar header; info = {lo, hi, start, end} (start/end ~0: no header /
 *      malformed on the speculative chain).
 *   2. The ranks exchange info and fix the true chain in rank order: pos(0) = 0,
 *      pos(r+1) = the true end of range r, which is info.end when info.start == pos(r) (a
 *      walk from a group position is deterministic); otherwise rank r calls
 *      tsg_layer_range_sync(pos(r)) and publishes its end (trivy_amd/shard.py:layer_chain).
 *      Every rank calls tsg_layer_range_sync with its pos before steps 3-4.
 *   3. tsg_layer_range_dirs: the dirs this range adds to the walker's skipDirs (tar.go:62-66),
 *      NUL-terminated, in walk order; they are handed to the later ranks.
 *   4. tsg_layer_range_pack: tar.go:45-84 over the range's entries with the earlier ranks'
 *      skip dirs first, then Required / IsBinary and the pack.  opq / wh are the range's own.
 * The union over ranks equals tsg_layer_pack's batch; an archive error on the true chain is
 * returned by the sync of the range holding it, as one sequential walk would report it. */
typedef struct tsg_layer_range tsg_layer_range;
int tsg_layer_range_walk(const uint8_t* tar, uint64_t tar_len, uint32_t rank, uint32_t world,
                         tsg_layer_range** out, uint64_t info[4]);
int tsg_layer_range_sync(tsg_layer_range* range, uint64_t pos, uint64_t* end);
int tsg_layer_range_dirs(tsg_layer_range* range, const char* const* skip_dirs, uint32_t n_skip_dirs,
                         const char** out, uint64_t* out_len);
int tsg_layer_range_pack(const tsg_ruleset* rs, const tsg_layer_range* range,
                         const char* const* skip_files, uint32_t n_skip_files,
                         const char* const* skip_dirs, uint32_t n_skip_dirs,
                         const char* const* prior_dirs, uint32_t n_prior_dirs,
                         const char* config_path, tsg_layer** out);
void tsg_layer_range_free(tsg_layer_range* range);
/* Filesystem ingest (configs[0], trivy fs): replaces walker.FS.Walk (pkg/fanal/walker/fs.go:25-63)
 * + the fs artifact's relative paths (pkg/fanal/artifact/local/fs.go:83-100) + Required +
 * IsBinary; files are read in parallel and packed in path order (paths relative to root, no
 * "/" prefix).  Result in the same tsg_layer form (no whiteouts). */
int tsg_fs_pack(const tsg_ruleset* rs, const char* root, const char* const* skip_files,
                uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                const char* config_path, tsg_layer** out);
/* One rank's share of a tree (configs[0] over several GPUs, one process each): every rank
 * lists the tree (no file opened), the listed files in path order are cut into `world`
 * contiguous runs of about equal bytes, and only this rank's run is read, IsBinary-gated
 * and packed.  Concatenated in rank order the shards are tsg_fs_pack's batch; walked is the
 * whole tree's. */
int tsg_fs_pack_shard(const tsg_ruleset* rs, const char* root, const char* const* skip_files,
                      uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                      const char* config_path, uint32_t rank, uint32_t world, tsg_layer** out);
/* Ingest straight into a pinned slot: tsg_layer_pack / tsg_layer_range_pack /
 * tsg_fs_pack whose kept files are written into a slot acquired from ctx instead of pageable
 * memory, so no second copy precedes the upload: a layer's files are copied once, tar ->
 * slot, and a tree's files are read straight into it (pread).  The rule set is ctx's.  On
 * success *slot_id is the caller's, as after tsg_slot_acquire: the slot's offsets and paths
 * are filled in, so tsg_slot_submit(ctx, *slot_id, view.nfiles) scans it, and
 * tsg_slot_release gives it back; the tsg_layer's view (tsg_layer_get) points into the slot
 * and is valid until then.  Waits, like tsg_slot_acquire, while every slot is busy. */
int tsg_layer_pack_slot(tsg_ctx* ctx, const uint8_t* tar, uint64_t tar_len,
                        const char* const* skip_files, uint32_t n_skip_files,
                        const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                        uint32_t* slot_id, tsg_layer** out);
int tsg_layer_range_pack_slot(tsg_ctx* ctx, const tsg_layer_range* range,
                              const char* const* skip_files, uint32_t n_skip_files,
                              const char* const* skip_dirs, uint32_t n_skip_dirs,
                              const char* const* prior_dirs, uint32_t n_prior_dirs,
                              const char* config_path, uint32_t* slot_id, tsg_layer** out);
int tsg_fs_pack_slot(tsg_ctx* ctx, const char* root, const char* const* skip_files,
                     uint32_t n_skip_files, const char* const* skip_dirs, uint32_t n_skip_dirs,
                     const char* config_path, uint32_t* slot_id, tsg_layer** out);
/* One call per layer / tree, pipelined (what a per-layer goroutine binds,
 * pkg/fanal/artifact/image/image.go:210-234): the walk and gates of tsg_layer_pack /
 * tsg_fs_pack, then the kept files cut in walk order into pieces of about the context's slot
 * size; each piece is written straight into a pinned slot and submitted while the next one
 * is written, so ingest, upload, kernels and host resolution overlap.  *out holds one record
 * per kept file in the order of *layer's paths (tsg_result format); *layer carries the paths,
 * offsets, opq, wh and walked count (its data view is NULL: the bytes lived in the slots).
 * tsg_fs_scan opens no file during its walk: every file that passes Required is listed with
 * its lstat size and read straight into its place in a piece; a file that is binary
 * (IsBinary on the bytes read) or cannot be opened is scanned along and then left out of
 * *out and *layer, which therefore equal tsg_fs_pack's batch and its scan. */
int tsg_layer_scan(tsg_ctx* ctx, const uint8_t* tar, uint64_t tar_len,
                   const char* const* skip_files, uint32_t n_skip_files,
                   const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                   tsg_layer** layer, tsg_result** out);
int tsg_fs_scan(tsg_ctx* ctx, const char* root, const char* const* skip_files, uint32_t n_skip_files,
                const char* const* skip_dirs, uint32_t n_skip_dirs, const char* config_path,
                tsg_layer** layer, tsg_result** out);
void tsg_layer_free(tsg_layer* layer);

#ifdef __cplusplus
}
#endif
#endif /* TRIVY_SECRET_H */

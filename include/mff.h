/*
 * mff.h — C ABI of libmff.so, the MI355X (gfx950) minute-factor engine.
 *
 * The reference (C-X-Lu/Replication-of-Minute-Frequency-Factor) has no FFI: its
 * operator API is a Python callable, `calculate_method(df) -> df`, handed to
 * `MinFreqFactor.cal_exposure_by_min_data` (MinuteFrequentFactorCICC.py:50-55) and
 * invoked per day file at MinuteFrequentFactorCICC.py:22.  Each entry point below
 * replaces one piece of that path; the reference interface it replaces is cited on
 * every declaration.  INTEGRATION.md shows the ctypes binding a maintainer adds.
 *
 * Conventions
 *  - All pointers are DEVICE pointers owned by the caller (the library never
 *    allocates or frees caller memory).  Host pointers are marked `host`.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every call
 *    is asynchronous on that stream; none synchronises, allocates, or copies, so a
 *    caller may capture them into a hipGraph.
 *  - Return 0 on success, negative on error; mff_last_error() gives a thread-local
 *    message.  No C++ exception crosses this ABI.
 *  - Panel layout: field planes open/high/low/close float32 and volume uint32 (shares),
 *    each [D][S][240] (day, stock, minute 0..239 = 09:30..11:29, 13:00..14:59); presence
 *    mask uint32 [D][S][8], bit (m % 32) of word (m / 32) set when bar m exists.
 *    Prices finite > 0; volume 0 <= v <= MFF_VOLUME_MAX (the all-ones word is the sorts'
 *    absent-bar key).  Values of absent bars are don't-care.
 *  - Output layout: val float64 [rows][D][S], state uint8 [rows][D][S] with
 *    0 = ABSENT (the reference emits no row), 1 = NULL (polars null),
 *    2 = VALUE (may be NaN / +-inf).
 */
#ifndef MFF_H
#define MFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFF_NUM_FACTORS 58
#define MFF_STATE_ABSENT 0
#define MFF_STATE_NULL 1
#define MFF_STATE_VALUE 2

/* stage 2 methods, MinuteFrequentFactorCICC.py:190-238 */
#define MFF_ROLL_O 0   /* identity            MF:190-198 */
#define MFF_ROLL_M 1   /* rolling_mean        MF:199-209 */
#define MFF_ROLL_Z 2   /* (x-mean)/std(ddof0) MF:210-227 */
#define MFF_ROLL_STD 3 /* rolling_std(ddof0)  MF:228-238 */

/* stage 3 kinds */
#define MFF_XS_Z 0
#define MFF_XS_RANK 1

int mff_version(void);
const char* mff_last_error(void);
int mff_num_factors(void);
/* name of factor `id` (reference column name, e.g. "mmt_pm"); NULL if out of range */
const char* mff_factor_name(int id);

/* mff_ingest_rows volume column types */
#define MFF_VOLUME_F64 0
#define MFF_VOLUME_I64 1
#define MFF_VOLUME_F32 2
#define MFF_VOLUME_I32 3

/* mff_ingest_rows counters (uint32 errors[5]) */
#define MFF_INGEST_ERR_INDEX 0  /* stock / day index outside [0,S) x [0,D): row skipped */
#define MFF_INGEST_ERR_TIME 1   /* time off the 240-bar grid: row skipped (not an error: the
                                   caller lists the stock-day in the row set) */
#define MFF_INGEST_ERR_DUP 2    /* (stock, day, minute) already present (the same) */
#define MFF_INGEST_ERR_PRICE 3  /* open/high/low/close not finite > 0 */
#define MFF_INGEST_ERR_VOLUME 4 /* volume not integral in [0, MFF_VOLUME_MAX] */
#define MFF_VOLUME_MAX 4294967294u /* 2^32 - 2 shares per bar */

/*
 * Ingest: long day-frame rows -> dense panel.
 * Replaces: the per-file `pl.read_parquet` hand-off (MinuteFrequentFactorCICC.py:22)
 * and the time -> minute map minute_in_trade (CM:98-106).  Row i: stock[i] / day[i]
 * (dense indices into the caller's sorted code / date universes, int32), time[i]
 * (HHMMSSmmm, int64), the four prices (float64) and volume (volume_kind).  Writes the
 * four fp32 price planes and the u32 volume plane of `bars` [5][D][S][240] (4 B per bar
 * each; the caller views the volume plane as uint32) at (day, stock, minute), ORs the presence
 * bit into `valid` [D][S][8]; `valid` and `errors` (uint32[5], MFF_INGEST_ERR_*) must be
 * zeroed by the caller before the first call into a panel, so a panel may be filled by
 * several calls (day-file batches).  Contract violations are counted, never trapped;
 * the caller reads `errors` and rejects the panel if any is non-zero.
 */
int mff_ingest_rows(const int32_t* stock, const int32_t* day, const int64_t* time,
                    const double* open, const double* high, const double* low,
                    const double* close, const void* volume, int volume_kind, int64_t nrows,
                    int S, int D, float* bars, uint32_t* valid, uint32_t* errors, void* stream);

/*
 * Stage 1: the per-(stock, day) factor kernels.
 * Replaces: every `cal_<name>(df)` of MinuteFrequentFactorCalculateMethodsCICC.py
 * (CM:12-1406) applied per day file by `_process_single_file`
 * (MinuteFrequentFactorCICC.py:17-25), for D days x S stocks at once.
 * factor_ids (host, nf entries): catalogue ids in output-row order.
 * pdf_query: float64 [5][D][S] workspace, required when any doc_pdf* id is requested
 * (the doc_pdf values are then produced by mff_pdf_* below), else may be NULL.
 * pdf_levels: mff_pdf_levels_bytes(S, D) bytes, required with doc_pdf (else NULL): per
 * day, every stock-day's price levels as (key c_last/c_level, total-order u64; bars at
 * the level, u8) that mff_pdf_count / mff_pdf_rank_local bin against the sorted queries
 * (filled and counted by the call itself), in two lists split at a key the library sets
 * per call (the mean median doc_pdf query of earlier calls on the device; 1.0 before
 * any: any key gives the same ranks): the keys below it from the front of the day's
 * S*256 slots (at most 255 levels per stock-day: MFF_ROWS_MAX), the others from the back, with the per-day counts (u32 pairs A, B = one
 * u64 counter per day) and the split key u64 in front.
 * workspace: mff_stage1_workspace_bytes(S, D) bytes of device scratch (the list of
 * stock-days the exact general path finishes; zeroed by the call itself).
 * Environment MFF_STAGE1_IMPL=w64 selects the wave-per-stock-day kernel for everything.
 */
size_t mff_stage1_workspace_bytes(int S, int D);
/* mff_stage1 in two calls with the same arguments: part 1 = the LVL/PDF group (
 * doc_pdf levels and queries, exact list), part 2 = ORD + the serial families.  Once part 1 is
 * done the mff_pdf_* phases may run on another stream, concurrently with part 2.
 * part 3 = mff_stage1.  part 4 = the high / low serial families (OLS, MOMH) alone, which
 * depend on no other launch (any stream, any time); part 10 / 11 = part 2 / 3 without them.
 * part 17 = part 1 without the exact list kernel, part 32 = that kernel alone (after part
 * 17, before the mff_pdf_* phases and before the LVL/PDF rows are read; part 2 need not
 * wait for it).  part 64 = part 1's prologue alone (zeroes the doc_pdf level-list counts,
 * sets the split key, zeroes the exact-list count: mff_stage1_rows phase 1 may start after
 * it), part 129 / 145 = part 1 / 17 without that prologue. */
int mff_stage1_part(const float* open, const float* high, const float* low,
                    const float* close, const uint32_t* volume, const uint32_t* valid,
                    int S, int D, const int32_t* factor_ids /* host */, int nf,
                    double* val, uint8_t* state, double* pdf_query, void* pdf_levels,
                    void* workspace, void* stream, int part);
size_t mff_pdf_levels_bytes(int S, int D);
int mff_stage1(const float* open, const float* high, const float* low,
               const float* close, const uint32_t* volume, const uint32_t* valid,
               int S, int D, const int32_t* factor_ids /* host */, int nf,
               double* val, uint8_t* state, double* pdf_query, void* pdf_levels,
               void* workspace, void* stream);

/*
 * Row set: the stock-days computed from their own rows instead of the 240-bar grid.
 * A stock-day is listed when a row of it holds a polars null (open / high / low / close /
 * volume) or sits off the grid (a time that is not a 09:30-11:29 / 13:00-14:59 minute:
 * a 09:25 or 15:00 bar, end-labelled bars, seconds) or shares its time with another row.
 * The panel's `valid` mask holds zeros for a listed stock-day except bit 31 of word 7
 * (MFF_ROWS_LISTED: bars end at 239), so the grid kernels see it ABSENT and store nothing
 * for it -- mff_stage1_rows writes all its rows and may run on another stream at the same
 * time.  A stock-day listed only for nulls on grid bars (its rows are its present bars)
 * may instead keep its presence bits in `valid` and carry MFF_ROWS_KEEP plus the null
 * fields (bit MFF_ROWS_NULL_SHIFT + i: field i = open, high, low, close, volume holds a
 * null on some bar) in word 7 AND in the `reserved` word of its first row: then a family
 * that reads none of those fields comes from the grid kernels (its values do not depend
 * on the null fields) and mff_stage1_rows computes only the families that read one.
 * The row set carries every one of its rows:
 *   rs_sd int32 [K]     d*S + s, ascending
 *   rs_off int32 [K+1]  rows of stock-day i: rs_rows[rs_off[i] .. rs_off[i+1]), at most
 *                       MFF_ROWS_MAX, in (time, frame) order (rows at one time
 *                       keep their frame order), minute_in_trade (CM:98-106) non-decreasing
 *   rs_rows MffRow [rs_off[K]]  time HHMMSSmmm in [0, 240000000), prices fp32, volume u32
 *                       shares, nulls = bit i set when field i (open, high, low, close,
 *                       volume) is null (its value is then don't-care), reserved = 0 except
 *                       on a kept stock-day's first row (MFF_ROWS_KEEP | null fields, as in
 *                       its `valid` word 7)
 */
#define MFF_ROWS_MAX 255
#define MFF_ROWS_LISTED 0x80000000u /* valid[d][s][7] of a listed stock-day */
#define MFF_ROWS_KEEP 0x40000000u   /* grid bars kept; only the families reading a null field listed */
#define MFF_ROWS_NULL_SHIFT 24      /* bits 24..28: the fields holding a null (with MFF_ROWS_KEEP) */
typedef struct MffRow {
  int32_t time;
  float open, high, low, close;
  uint32_t volume;
  uint32_t nulls;
  uint32_t reserved;
} MffRow; /* 32 B */

/*
 * Stage 1 of the row set.  Replaces the same `cal_*` calls (CM:12-1406) on those rows:
 * polars' null rules (only cal_liq_amihud_1min fills a null volume with 0, CM:743-744;
 * first()/last() return the null, CM:799, 829; sums / moments skip it; pl.corr drops the
 * pair, CM:841-931; pct_change forward-fills, CM:745, 861-866; top_k prefers non-null
 * values, CM:393-471; rank() leaves a null key unranked, CM:1016 -- the rules N1-N11 / C8
 * of oracle/mff_oracle.py), the time filters on each row's own time (CM:18-84, 770-815,
 * 1212-1387) and the 50-minute OLS windows over minute_in_trade (CM:98-129).
 * phase 1: doc_pdf queries + the stock-days' price levels appended to pdf_levels (call
 *          after mff_stage1_part 1 / 17 and before mff_pdf_sort);
 * phase 2: every other requested row (call after the stage-1 calls that write those rows);
 * phase 3: both (e.g. after mff_stage1 when no doc_pdf row is requested).
 */
int mff_stage1_rows(int S, int D, const int32_t* rs_sd, const int32_t* rs_off, const MffRow* rs_rows, int K,
                    const int32_t* factor_ids /* host */, int nf, double* val, uint8_t* state,
                    double* pdf_query, void* pdf_levels, int phase, void* stream);
/*
 * Grid stock-days -> rows (e.g. to list stock-days of a device-built panel): for each of
 * the K stock-days sd[K], its present bars in minute order, time = the bar's start label,
 * null bits from null_bits uint32 [K][5][8] (the `valid` bit layout per field; NULL =
 * none).  Count mode (rows == NULL): counts int32 [K] = rows per stock-day (the caller
 * turns them into off [K+1]); else the rows are written at rows[off[i] ...].
 */
int mff_rows_from_panel(const float* open, const float* high, const float* low, const float* close,
                        const uint32_t* volume, const uint32_t* valid, int S, int D, const int32_t* sd,
                        const uint32_t* null_bits, int K, const int32_t* off, int32_t* counts, MffRow* rows,
                        void* stream);

/*
 * Multi-day frame semantics of the four factors whose reference windows run over('code')
 * only: liq_amihud_1min (CM:745-746 pct_change over code), corr_prvr (CM:855-867),
 * trade_bottom20retRatio (CM:1212-1216 volume.sum().over('code')) and
 * trade_bottom50retRatio (CM:1233-1241).  The reference driver calls cal_* per day file
 * (MinuteFrequentFactorCICC.py:22), where they are per-day; a cal_* handed a frame of
 * several dates reaches across them.  Given the panel of such a frame (days = the frame's
 * dates, rows of a code in (date, time) order) and stage 1's output rows, this call
 * overwrites the rows of those four factors (when present in factor_ids) with the frame
 * semantics: the first bar of a day compares with the code's last close of the previous
 * day, and the 14:40+ / 14:10+ volume share uses the code's total over the whole frame.
 * open may be NULL unless a trade_bottom* row is requested.  rs_sd / rs_off / rs_rows (the
 * panel's row set, K = 0 and NULLs when it has none) give the listed stock-days' rows: a
 * null volume is 0 for the Amihud sum (CM:743-744) and filtered out by volume != 0
 * (CM:855), a null close is forward-filled by pct_change (CM:745, 861), the tail windows
 * test each row's own time (CM:1212, 1233).
 */
int mff_stage1_frame(const float* open, const float* close, const uint32_t* volume,
                     const uint32_t* valid, int S, int D, const int32_t* rs_sd, const int32_t* rs_off,
                     const MffRow* rs_rows, int K, const int32_t* factor_ids /* host */, int nf,
                     double* val, uint8_t* state, void* stream);

/*
 * doc_pdf60..95 frame-wide rank (CM:1015-1017: `.rank()` over ALL rows of the day
 * frame, every code).  Device phases; each works on days [d0, d0+nd) of arrays laid
 * out over all D days.
 *   sort:     queries of R ranks, float64 [R][5][D][S_all] (NaN = none; each rank's
 *             [5][D][S_loc] padded to S_all with NaN)
 *             -> q_sorted uint64 [nd][M], M = R*5*S_all (total-order keys; any M: beyond
 *             32768 per day the sort finishes with global merge passes)
 *   count:    this rank's keys c_last/c_b (from stage 1's pdf_levels: one key per
 *             distinct close of a stock-day, weighted by its bar count) against q_sorted
 *             -> counts uint32 [nd][M] = 2 n_less + n_eq over local keys (the
 *             average rank n_less + (n_eq + 1) / 2 is linear in it)
 *   [R > 1: the caller sums `counts` over ranks (reduce-scatter to each day's owner, or
 *    an all-reduce), see INTEGRATION.md]
 *   finalize: own queries [5][D][S_loc] -> val/state rows pdf_rows[5] (host, -1 = skip),
 *             looking each query up in the day's sorted list and the summed counts
 *   origin_counts: day-owner side of the reduce-scatter exchange: the summed counts of
 *             the owned days at each query of q_all [R][5][D][S_all] (days [d0, d0+nd)),
 *             written in that origin layout -> out uint32 [R][5][nd][S_all] (0 for NaN);
 *             q_sorted / counts may be the deduplicated lists [nd][M] (M <= R*5*S_all,
 *             each day's distinct keys padded with ~0: the counts of a value sit at its
 *             first position);
 *             one all_to_all then hands every rank its own queries' counts
 *   finalize_own: own queries [5][D][S_loc] with their counts in the same layout
 *             (2 n_less + n_eq summed over ranks) -> val/state (rank (c + 1) / 2)
 *   rank_local: count + finalize in one pass, for a single rank (R = 1: no exchange)
 * workspace: mff_pdf_workspace_bytes(S_loc, R, nd) bytes of device scratch (sort).
 */
size_t mff_pdf_workspace_bytes(int S_loc, int R, int nd);
int mff_pdf_sort(const double* q_all, int R, int S_all, int D, int d0, int nd,
                 uint64_t* q_sorted, void* workspace, void* stream);
int mff_pdf_count(const void* pdf_levels, int S_loc, int D, int d0, int nd,
                  const uint64_t* q_sorted, int M, uint32_t* counts, void* workspace,
                  void* stream);
/* Frame-wide count (one cal_doc_pdf* call on a frame holding several dates: `.rank()`
 * at CM:1015-1017 ranks every row of every date).  The D days' queries are sorted as ONE
 * list (mff_pdf_sort with the [5][D][S] queries viewed as [5][1][D*S]); every day's level
 * keys are counted against it and their words 2 n_less + n_eq ADDED to counts uint32 [M]
 * (zeroed by the caller); mff_pdf_finalize with S_loc = D*S, D = 1 then writes the ranks.
 * Requires 240*S*D < 2^31 and M <= 2^24. */
int mff_pdf_count_frame(const void* pdf_levels, int S, int D, const uint64_t* q_sorted, int M,
                        uint32_t* counts, void* stream);
int mff_pdf_finalize(const double* q_local, const uint64_t* q_sorted,
                     const uint32_t* counts, int S_loc, int D, int d0, int nd, int M,
                     const int32_t* pdf_rows /* host, 5 entries, -1 = skip */,
                     double* val, uint8_t* state, void* stream);
int mff_pdf_origin_counts(const double* q_all, int R, int S_all, int D, int d0, int nd,
                          const uint64_t* q_sorted, const uint32_t* counts, int M, uint32_t* out,
                          void* stream);
int mff_pdf_finalize_own(const double* q_local, const uint32_t* own_counts, int S_loc, int D,
                         const int32_t* pdf_rows /* host, 5 entries, -1 = skip */, double* val,
                         uint8_t* state, void* stream);
int mff_pdf_rank_local(const void* pdf_levels, const double* q_local,
                       int S, int D, int d0, int nd, const uint64_t* q_sorted, int M,
                       const int32_t* pdf_rows /* host, 5 entries */, double* val,
                       uint8_t* state, void* stream);

/*
 * Stage 2: N-day rolling post-processing over present days, per stock.
 * Replaces: MinFreqFactor.cal_final_exposure(frequency=N, method, mode='days')
 * (MinuteFrequentFactorCICC.py:187-240).  rows = number of factor rows.
 * Any N >= 1, like the reference's `frequency: int` (MF:188-189, 205).
 */
int mff_stage2(const double* val, const uint8_t* state, int rows, int D, int S,
               int N, int method, double* out_val, uint8_t* out_state, void* stream);

/*
 * Calendar resampling, mode='calendar' of cal_final_exposure (MinuteFrequentFactorCICC.py:
 * 130-186; the reference raises there: group_by_dynamic without index_column, MF:145 —
 * this is the build's definition): per stock and calendar window p (days
 * [period_start[p], period_start[p+1]), period_start int32 [P+1] device, date-sorted),
 * over the window's rows: 'o' last value (null if the last row is null), 'm' mean,
 * 'std' std (ddof=1), 'z' (last - mean) / std; nulls skipped, NaN propagates.
 * Output [P][S]: ABSENT where the stock has no row in the window.
 */
int mff_calendar(const double* val, const uint8_t* state, const int32_t* period_start, int D,
                 int S, int P, int method, double* out_val, uint8_t* out_state, void* stream);

/*
 * Stage 3: per-day cross-sectional z-score (ddof=1) or average rank over stocks with
 * state VALUE and non-NaN value.  No single reference function; closest semantics
 * Factor.py:99-105 (coverage), :163-186 (per-date Pearson / Spearman), :285-291 (qcut).
 * z-score, multi-GPU: mff_xs_moments per rank -> all-gather [R][rows][D][3] ->
 * mff_xs_zscore.  rank: all-gather values/states [R][rows][D][S_all] (every rank's
 * columns padded to S_all with ABSENT) -> mff_xs_rank.
 */
int mff_xs_moments(const double* val, const uint8_t* state, int rows, int D, int S,
                   double* moments /* [rows][D][3]: n, mean, M2 */, void* stream);
int mff_xs_zscore(const double* val, const uint8_t* state, int rows, int D, int S,
                  const double* moments_all, int R, double* out_val,
                  uint8_t* out_state, void* stream);
/* Single-rank z in one pass (same result contract as moments + zscore with R = 1):
 * one workgroup per (row, day) holds the column in registers; S <= max_stocks(). */
int mff_xs_zscore_local(const double* val, const uint8_t* state, int rows, int D, int S,
                        double* out_val, uint8_t* out_state, void* stream);
int mff_xs_zscore_local_max_stocks(void);
size_t mff_xs_rank_workspace_bytes(int rows, int D, int S_all, int R);
int mff_xs_rank(const double* val, const uint8_t* state, int rows, int D, int S_loc,
                const double* val_all, const uint8_t* state_all, int R, int S_all,
                double* out_val, uint8_t* out_state, void* workspace, void* stream);

/*
 * Factor IC / rank-IC test.  Replaces Factor.ic_test
 * (Factor.py:127-229).  Inputs are dense [D][S] (val, state) like stage 1's output rows.
 * mff_future_return: Factor.py:142-162 — per stock over its present days,
 *   fut = exp(sum of log(1 + pct) over the next N present days) - 1, NULL unless N such
 *   days exist with no null among them (rolling_sum min_samples=N, then shift(-N)).
 *   Any N >= 1 (Factor.py:149 takes any future_days).
 * mff_ic_pairs: the pair set of pl.corr (Factor.py:165-183): x VALUE and not NaN (the
 *   is_nan filter), y VALUE; writes [2][D][S] rows (x, y) with state VALUE on pairs, else
 *   ABSENT.  Feed them to mff_ic_moments (IC) or first to mff_xs_rank (rank IC).
 * mff_ic_moments: per day, the local pair moments partial [D][6] = (n, mean_x, mean_y,
 *   Cxx, Cyy, Cxy) over pairs whose two states are VALUE.
 * mff_ic_finalize: combine the R stock shards' partials [R][D][6] (all-gathered) and
 *   write ic [D] = Cxy / sqrt(Cxx Cyy), NaN when n < 2 or the denominator is 0.
 */
int mff_future_return(const double* pct, const uint8_t* state, int D, int S, int N,
                      double* out_val, uint8_t* out_state, void* stream);
int mff_ic_pairs(const double* x_val, const uint8_t* x_state, const double* y_val,
                 const uint8_t* y_state, int D, int S, double* pair_val, uint8_t* pair_state,
                 void* stream);
int mff_ic_moments(const double* pair_val, const uint8_t* pair_state, int D, int S,
                   double* partial, void* stream);
int mff_ic_finalize(const double* partial_all, int R, int D, double* ic, void* stream);

/*
 * Factor group back-test.  Replaces Factor.group_test
 * (Factor.py:231-350).  Exposure / pct_change / weight rows are dense [D][S] (val, state).
 * mff_bt_qcut: per date, G quantile groups of the non-null non-NaN exposures of all
 *   ranks (val_all/state_all [R][D][S_all], each rank's columns padded with ABSENT):
 *   pandas-qcut edges (linear quantiles, duplicate edges dropped) -> group int8 [D][S_loc]
 *   in 0..G-1, -1 = null.  workspace: mff_bt_qcut_workspace_bytes bytes.  G <= 63.
 * mff_bt_periods: per stock over the dates (period_of [D] int32, non-decreasing, every
 *   period 0..P-1 present): per period the return prod(1 + pct) - 1 over the exposure
 *   rows with non-null pct, and the group / weight of the previous period the stock held
 *   (shift(1).over('code')) -> p_ret f64, p_group int8 (-1 = null), p_weight f64 +
 *   p_weight_state u8, all [P][S].  weight / weight_state NULL = equal weights.
 * mff_bt_reduce: per (period, group) over local stocks -> partial [P][G][4] = (count,
 *   sum ret, sum w, sum w*ret).
 * mff_bt_finalize: sum the R ranks' partials [R][P][G][4] -> ret [P][G] = mean ret, or
 *   (weighted) sum w*ret / sum w (0 when sum w == 0); present [P][G] u8 = count > 0.
 */
size_t mff_bt_qcut_workspace_bytes(int D, int S_all, int R);
int mff_bt_qcut(const double* val, const uint8_t* state, int D, int S_loc, const double* val_all,
                const uint8_t* state_all, int R, int S_all, int G, int8_t* group, void* workspace,
                void* stream);
int mff_bt_periods(const uint8_t* x_state, const int8_t* group, const double* pct,
                   const uint8_t* pct_state, const double* weight, const uint8_t* weight_state,
                   const int32_t* period_of, int D, int S, int P, double* p_ret, int8_t* p_group,
                   double* p_weight, uint8_t* p_weight_state, void* stream);
int mff_bt_reduce(const double* p_ret, const int8_t* p_group, const double* p_weight,
                  const uint8_t* p_weight_state, int P, int S, int G, double* partial, void* stream);
int mff_bt_finalize(const double* partial_all, int R, int P, int G, int weighted, double* ret,
                    uint8_t* present, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MFF_H */

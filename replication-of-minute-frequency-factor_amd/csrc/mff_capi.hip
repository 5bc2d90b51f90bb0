// mff_capi.hip — library-wide C ABI: version, error slot, factor catalogue.
#include <stdarg.h>

#include "../../include/mff.h"
#include "mff_internal.h"

namespace mff {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

// reference order, MinuteFrequentFactorCalculateMethodsCICC.py:12-1381
const char* const kFactorNames[NF] = {
    "mmt_pm", "mmt_last30", "mmt_paratio", "mmt_am", "mmt_between",
    "mmt_ols_qrs", "mmt_ols_corr_square_mean", "mmt_ols_corr_mean",
    "mmt_ols_beta_mean", "mmt_ols_beta_zscore_last",
    "mmt_top50VolumeRet", "mmt_bottom50VolumeRet", "mmt_top20VolumeRet",
    "mmt_bottom20VolumeRet",
    "vol_volume1min", "vol_range1min", "vol_return1min", "vol_upVol", "vol_upRatio",
    "vol_downVol", "vol_downRatio",
    "shape_skew", "shape_kurt", "shape_skratio", "shape_skewVol", "shape_kurtVol",
    "shape_skratioVol",
    "liq_amihud_1min", "liq_closeprevol", "liq_closevol", "liq_firstCallR",
    "liq_lastCallR", "liq_openvol",
    "corr_prv", "corr_prvr", "corr_pv", "corr_pvd", "corr_pvl", "corr_pvr",
    "doc_kurt", "doc_skew", "doc_std", "doc_pdf60", "doc_pdf70", "doc_pdf80",
    "doc_pdf90", "doc_pdf95", "doc_vol10_ratio", "doc_vol5_ratio", "doc_vol50_ratio",
    "trade_bottom20retRatio", "trade_bottom50retRatio", "trade_headRatio",
    "trade_tailRatio", "trade_top20retRatio", "trade_top50retRatio",
    "trade_topNeg20retRatio", "trade_topPos20retRatio",
};



static_assert([] {  // the table in mff_internal.h and the device lookup agree
  for (int f = 0; f < NF; ++f)
    if (kFactorFamily[f] != kFamOf(f)) return false;
  return true;
}(), "kFamOf (device) disagrees with kFactorFamily");

}  // namespace mff

extern "C" {

int mff_version(void) { return 1; }
const char* mff_last_error(void) { return mff::g_err; }
int mff_num_factors(void) { return mff::NF; }
const char* mff_factor_name(int id) {
  return (id >= 0 && id < mff::NF) ? mff::kFactorNames[id] : nullptr;
}

}  // extern "C"

// probe.hpp — host pre-screen of one image (dino_probe / dino_probe_spans /
// dino_gather_probe / the native feed): the device parser run on the CPU.
#pragma once

#include "jpeg_parse.hpp"
#include "plan.hpp"
#include "progressive.hpp"

namespace dino {

constexpr int32_t kMaxImageDim = 65535;

// One image of dino_probe / dino_probe_spans / dino_gather_probe: its info row and workspace bytes.
inline void probe_one(const uint8_t* p, int64_t len, bool raw, int32_t max_image_dim, const dino_aug_config* cfg,
               ScanRec* scans, int32_t* info_row, int64_t* ws, int64_t* aws) {
  ImgDesc d;
  if (len <= 0) {
    d.status = DINO_IMG_CORRUPT;
    d.width = d.height = d.ncomp = 0;
  } else {
    parse_jpeg(p, len, max_image_dim, &d, raw);
    if (d.status == DINO_IMG_OK && d.kind == 1) {
      HostMarkerFinder find;
      if (prog_walk(p, len, &d, scans, find) == DINO_IMG_OK) {
        // k_pwalk's table slots: more distinct tables than the region holds -> Pillow
        int32_t slot_off[kPMaxTabs];
        uint8_t slot_dc[kPMaxTabs];
        uint64_t ts[kMaxScans];
        if (prog_table_slots(scans, d.n_scans, slot_off, slot_dc, ts, kPMaxTabs) < 0) d.status = DINO_IMG_UNSUPPORTED;
      }
    }
  }
  if (info_row) {
    info_row[0] = d.status;
    info_row[1] = d.status == DINO_IMG_OK || d.status > 0 ? d.width : 0;
    info_row[2] = d.status == DINO_IMG_OK || d.status > 0 ? d.height : 0;
    info_row[3] = d.status == DINO_IMG_OK ? d.kind : -1;
  }
  if (d.status != DINO_IMG_OK) return;
  *ws += image_chunk_bytes(d).total();
  if (cfg) {
    for (int v = 0; v < cfg->n_global + cfg->n_local; ++v)
      *aws += view_scratch_bound(v < cfg->n_global ? cfg->global_size : cfg->local_size, d.width, d.height);
  }
}

}  // namespace dino

#pragma once
// fwd_g1: 1393 VALU, 1535 lines
#define MI_TW_BODY_FWD_G1(...) asm volatile(\
      "s_mov_b64 s[22:23], exec\n"\
      "s_add_u32 s78, %[g_lo], 0\n"\
      "s_addc_u32 s79, %[g_hi], 0\n"\
      "s_add_u32 s80, %[g_lo], 4096\n"\
      "s_addc_u32 s81, %[g_hi], 0\n"\
      "s_add_u32 s82, %[g_lo], 8192\n"\
      "s_addc_u32 s83, %[g_hi], 0\n"\
      "s_add_u32 s84, %[g_lo], 12288\n"\
      "s_addc_u32 s85, %[g_hi], 0\n"\
      "s_add_u32 s86, %[tw_lo], 0\n"\
      "s_addc_u32 s87, %[tw_hi], 0\n"\
      "s_add_u32 s88, %[tw_lo], 4096\n"\
      "s_addc_u32 s89, %[tw_hi], 0\n"\
      "s_add_u32 s90, %[tw_lo], 8192\n"\
      "s_addc_u32 s91, %[tw_hi], 0\n"\
      "s_add_u32 s92, %[tw_lo], 12288\n"\
      "s_addc_u32 s93, %[tw_hi], 0\n"\
      "s_mov_b32 s20, 0xaaaaaaaa\n"\
      "s_mov_b32 s21, 0xaaaaaaaa\n"\
      "global_load_dwordx2 v[64:65], %[l8], s[78:79] offset:0\n"\
      "global_load_dwordx2 v[66:67], %[l8], s[78:79] offset:512\n"\
      "global_load_dwordx2 v[68:69], %[l8], s[78:79] offset:1024\n"\
      "global_load_dwordx2 v[70:71], %[l8], s[78:79] offset:1536\n"\
      "global_load_dwordx2 v[72:73], %[l8], s[78:79] offset:2048\n"\
      "global_load_dwordx2 v[74:75], %[l8], s[78:79] offset:2560\n"\
      "global_load_dwordx2 v[76:77], %[l8], s[78:79] offset:3072\n"\
      "global_load_dwordx2 v[78:79], %[l8], s[78:79] offset:3584\n"\
      "global_load_dwordx2 v[80:81], %[l8], s[80:81] offset:0\n"\
      "global_load_dwordx2 v[82:83], %[l8], s[80:81] offset:512\n"\
      "global_load_dwordx2 v[84:85], %[l8], s[80:81] offset:1024\n"\
      "global_load_dwordx2 v[86:87], %[l8], s[80:81] offset:1536\n"\
      "global_load_dwordx2 v[88:89], %[l8], s[80:81] offset:2048\n"\
      "global_load_dwordx2 v[90:91], %[l8], s[80:81] offset:2560\n"\
      "global_load_dwordx2 v[92:93], %[l8], s[80:81] offset:3072\n"\
      "global_load_dwordx2 v[94:95], %[l8], s[80:81] offset:3584\n"\
      "global_load_dwordx2 v[96:97], %[l8], s[82:83] offset:0\n"\
      "global_load_dwordx2 v[98:99], %[l8], s[82:83] offset:512\n"\
      "global_load_dwordx2 v[100:101], %[l8], s[82:83] offset:1024\n"\
      "global_load_dwordx2 v[102:103], %[l8], s[82:83] offset:1536\n"\
      "global_load_dwordx2 v[104:105], %[l8], s[82:83] offset:2048\n"\
      "global_load_dwordx2 v[106:107], %[l8], s[82:83] offset:2560\n"\
      "global_load_dwordx2 v[108:109], %[l8], s[82:83] offset:3072\n"\
      "global_load_dwordx2 v[110:111], %[l8], s[82:83] offset:3584\n"\
      "global_load_dwordx2 v[112:113], %[l8], s[84:85] offset:0\n"\
      "global_load_dwordx2 v[114:115], %[l8], s[84:85] offset:512\n"\
      "global_load_dwordx2 v[116:117], %[l8], s[84:85] offset:1024\n"\
      "global_load_dwordx2 v[118:119], %[l8], s[84:85] offset:1536\n"\
      "global_load_dwordx2 v[120:121], %[l8], s[84:85] offset:2048\n"\
      "global_load_dwordx2 v[122:123], %[l8], s[84:85] offset:2560\n"\
      "global_load_dwordx2 v[124:125], %[l8], s[84:85] offset:3072\n"\
      "global_load_dwordx2 v[126:127], %[l8], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_lshlrev_b64 v[8:9], 16, v[96:97]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[98:99]\n"\
      "v_lshrrev_b32 v12, 16, v97\n"\
      "v_lshrrev_b32 v20, 16, v99\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mov_b32 v14, 0\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v96, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v97, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v67, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v96, s[36:37], v96, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[100:101]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[102:103]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[104:105]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[106:107]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[108:109]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[110:111]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[112:113]\n"\
      "v_lshrrev_b32 v28, 16, v101\n"\
      "v_lshrrev_b32 v36, 16, v103\n"\
      "v_lshrrev_b32 v44, 16, v105\n"\
      "v_lshrrev_b32 v52, 16, v107\n"\
      "v_lshrrev_b32 v60, 16, v109\n"\
      "v_lshrrev_b32 v12, 16, v111\n"\
      "v_lshrrev_b32 v20, 16, v113\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v80, v18\n"\
      "v_sub_co_u32_e64 v100, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v102, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v104, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v106, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v108, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v110, s[36:37], v78, v10\n"\
      "v_sub_co_u32_e64 v112, s[42:43], v80, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v81, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v101, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v103, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v105, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v107, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v109, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v111, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v113, s[44:45], v81, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v100, s[48:49], v100, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v102, s[54:55], v102, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v104, s[60:61], v104, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v106, s[66:67], v106, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v108, s[72:73], v108, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v110, s[36:37], v110, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v112, s[42:43], v112, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[114:115]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[116:117]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[118:119]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[120:121]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[122:123]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[124:125]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[126:127]\n"\
      "v_lshrrev_b32 v28, 16, v115\n"\
      "v_lshrrev_b32 v36, 16, v117\n"\
      "v_lshrrev_b32 v44, 16, v119\n"\
      "v_lshrrev_b32 v52, 16, v121\n"\
      "v_lshrrev_b32 v60, 16, v123\n"\
      "v_lshrrev_b32 v12, 16, v125\n"\
      "v_lshrrev_b32 v20, 16, v127\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v82, v26\n"\
      "v_sub_co_u32_e64 v114, s[48:49], v82, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v84, v34\n"\
      "v_sub_co_u32_e64 v116, s[54:55], v84, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v86, v42\n"\
      "v_sub_co_u32_e64 v118, s[60:61], v86, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v88, v50\n"\
      "v_sub_co_u32_e64 v120, s[66:67], v88, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v90, v58\n"\
      "v_sub_co_u32_e64 v122, s[72:73], v90, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_sub_co_u32_e64 v124, s[36:37], v92, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v94, v18\n"\
      "v_sub_co_u32_e64 v126, s[42:43], v94, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v83, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v115, s[50:51], v83, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v85, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v117, s[56:57], v85, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v87, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v119, s[62:63], v87, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v89, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v121, s[68:69], v89, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v91, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v123, s[74:75], v91, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v125, s[38:39], v93, v11, s[36:37]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v95, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v127, s[44:45], v95, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v114, s[48:49], v114, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v116, s[54:55], v116, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v118, s[60:61], v118, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v120, s[66:67], v120, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v122, s[72:73], v122, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v124, s[36:37], v124, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v126, s[42:43], v126, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v127, s[24:25], v127, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[80:81]\n"\
      "v_lshlrev_b64 v[16:17], 24, v[82:83]\n"\
      "v_lshrrev_b32 v12, 8, v81\n"\
      "v_lshrrev_b32 v20, 8, v83\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v82, s[42:43], v66, v18\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v80, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[44:45], v67, v19, s[42:43]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v82, s[42:43], v82, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v80, s[36:37], v80, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v12, s[36:37]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[112:113]\n"\
      "v_lshlrev_b32 v20, 8, v112\n"\
      "v_lshlrev_b64 v[24:25], 24, v[84:85]\n"\
      "v_lshlrev_b64 v[32:33], 24, v[86:87]\n"\
      "v_lshlrev_b64 v[40:41], 24, v[88:89]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[94:95]\n"\
      "v_lshrrev_b32 v28, 8, v85\n"\
      "v_lshrrev_b32 v36, 8, v87\n"\
      "v_lshrrev_b32 v44, 8, v89\n"\
      "v_lshrrev_b32 v52, 8, v91\n"\
      "v_lshrrev_b32 v60, 8, v93\n"\
      "v_lshrrev_b32 v12, 8, v95\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_sub_co_u32_e64 v84, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v86, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v78, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v96, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v85, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v87, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v97, s[44:45], v97, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v84, s[48:49], v84, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v86, s[54:55], v86, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v96, s[42:43], v96, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v20, s[42:43]\n"\
      "v_lshrrev_b64 v[24:25], 24, v[114:115]\n"\
      "v_lshrrev_b64 v[32:33], 24, v[116:117]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[118:119]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 24, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 24, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[126:127]\n"\
      "v_lshlrev_b32 v28, 8, v114\n"\
      "v_lshlrev_b32 v36, 8, v116\n"\
      "v_lshlrev_b32 v44, 8, v118\n"\
      "v_lshlrev_b32 v52, 8, v120\n"\
      "v_lshlrev_b32 v60, 8, v122\n"\
      "v_lshlrev_b32 v12, 8, v124\n"\
      "v_lshlrev_b32 v20, 8, v126\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v28, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_sub_co_u32_e64 v27, s[48:49], v27, v28\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[48:49]\n"\
      "v_addc_co_u32_e64 v26, s[50:51], v26, 0, s[48:49]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v29, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v104, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v106, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v108, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v110, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_sub_co_u32_e64 v98, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v100, s[54:55], v100, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v102, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v105, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v104, s[66:67], v104, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v107, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v106, s[72:73], v106, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v109, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v108, s[36:37], v108, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v111, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v110, s[42:43], v110, v18\n"\
      "v_subb_co_u32_e64 v99, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v101, s[56:57], v101, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v103, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v105, s[68:69], v105, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v107, s[74:75], v107, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v109, s[38:39], v109, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v111, s[44:45], v111, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v98, s[48:49], v98, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v100, s[54:55], v100, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v102, s[60:61], v102, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v104, s[66:67], v104, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v106, s[72:73], v106, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v108, s[36:37], v108, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v110, s[42:43], v110, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[116:117], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 12, v[72:73]\n"\
      "v_lshlrev_b64 v[16:17], 12, v[74:75]\n"\
      "v_lshrrev_b32 v12, 20, v73\n"\
      "v_lshrrev_b32 v20, 20, v75\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v72, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v74, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v73, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v75, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 28, v[88:89]\n"\
      "v_lshrrev_b32 v44, 4, v89\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v72, s[36:37], v72, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v74, s[42:43], v74, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshlrev_b64 v[48:49], 28, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 28, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 28, v[94:95]\n"\
      "v_lshlrev_b64 v[16:17], 4, v[104:105]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshrrev_b32 v52, 4, v91\n"\
      "v_lshrrev_b32 v60, 4, v93\n"\
      "v_lshrrev_b32 v12, 4, v95\n"\
      "v_lshrrev_b32 v20, 28, v105\n"\
      "v_lshlrev_b64 v[24:25], 12, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 12, v[78:79]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 20, v77\n"\
      "v_lshrrev_b32 v36, 20, v79\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v81, v43, s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v84, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v86, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v82, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v84, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v86, v10\n"\
      "v_sub_co_u32_e64 v104, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v85, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v87, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v85, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v87, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v105, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 4, v[106:107]\n"\
      "v_lshlrev_b64 v[32:33], 4, v[108:109]\n"\
      "v_lshlrev_b64 v[40:41], 4, v[110:111]\n"\
      "v_lshrrev_b32 v28, 28, v107\n"\
      "v_lshrrev_b32 v36, 28, v109\n"\
      "v_lshrrev_b32 v44, 28, v111\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v104, s[42:43], v104, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 12, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 12, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 12, v[126:127]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 20, v120\n"\
      "v_lshlrev_b32 v60, 20, v122\n"\
      "v_lshlrev_b32 v12, 20, v124\n"\
      "v_lshlrev_b32 v20, 20, v126\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v116, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v118, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v106, s[48:49], v98, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_sub_co_u32_e64 v108, s[54:55], v100, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_sub_co_u32_e64 v110, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v112, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v114, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v117, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v116, s[36:37], v116, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v119, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v118, s[42:43], v118, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v107, s[50:51], v99, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v109, s[56:57], v101, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v111, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v113, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v115, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v117, s[38:39], v117, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v119, s[44:45], v119, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v106, s[48:49], v106, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v108, s[54:55], v108, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v110, s[60:61], v110, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v112, s[66:67], v112, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v114, s[72:73], v114, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v116, s[36:37], v116, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v118, s[42:43], v118, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 6, v[68:69]\n"\
      "v_lshrrev_b32 v12, 26, v69\n"\
      "v_lshlrev_b64 v[16:17], 6, v[70:71]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 26, v71\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_lshlrev_b64 v[24:25], 22, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 22, v[78:79]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshrrev_b32 v28, 10, v77\n"\
      "v_lshrrev_b32 v36, 10, v79\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v68, s[36:37], v64, v10\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v66, v18\n"\
      "v_subb_co_u32_e64 v69, s[38:39], v65, v11, s[36:37]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshrrev_b64 v[56:57], 18, v[92:93]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_lshlrev_b32 v60, 14, v92\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 30, v[84:85]\n"\
      "v_lshlrev_b64 v[48:49], 30, v[86:87]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v68, s[36:37], v68, 0, s[38:39]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v44, 2, v85\n"\
      "v_lshrrev_b32 v52, 2, v87\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_lshrrev_b64 v[8:9], 18, v[94:95]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_lshlrev_b32 v12, 14, v94\n"\
      "v_lshlrev_b64 v[16:17], 18, v[100:101]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 14, v101\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v82, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v88, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v89, s[74:75], v89, v59, s[72:73]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v90, v10\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v88, s[72:73], v88, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v74, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v74, v34\n"\
      "v_sub_co_u32_e64 v84, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v91, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v90, v10\n"\
      "v_sub_co_u32_e64 v100, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v60, s[72:73]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v75, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v72, v26\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v75, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v85, s[62:63], v81, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v91, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v101, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 10, v[116:117]\n"\
      "v_lshlrev_b64 v[56:57], 10, v[118:119]\n"\
      "v_lshrrev_b32 v52, 22, v117\n"\
      "v_lshrrev_b32 v60, 22, v119\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v73, v27, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v84, s[60:61], v84, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v100, s[42:43], v100, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_lshrrev_b64 v[32:33], 30, v[108:109]\n"\
      "v_lshrrev_b64 v[40:41], 30, v[110:111]\n"\
      "v_lshrrev_b64 v[8:9], 6, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 6, v[126:127]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_lshlrev_b32 v36, 2, v108\n"\
      "v_lshlrev_b32 v44, 2, v110\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v12, 26, v124\n"\
      "v_lshlrev_b32 v20, 26, v126\n"\
      "v_lshlrev_b64 v[24:25], 18, v[102:103]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 14, v103\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v106, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v122, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v104, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v107, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v106, s[60:61], v106, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v116, s[66:67], v112, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_sub_co_u32_e64 v118, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v120, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v123, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v122, s[42:43], v122, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v105, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v107, s[62:63], v107, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v117, s[68:69], v113, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v119, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v121, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v123, s[44:45], v123, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v104, s[54:55], v104, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v106, s[60:61], v106, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v116, s[66:67], v116, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v118, s[72:73], v118, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v120, s[36:37], v120, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v122, s[42:43], v122, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[16:17], 19, v[70:71]\n"\
      "v_lshlrev_b64 v[8:9], 3, v[66:67]\n"\
      "v_lshrrev_b32 v20, 13, v71\n"\
      "v_lshrrev_b32 v12, 29, v67\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_sub_co_u32_e64 v66, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_subb_co_u32_e64 v67, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v66, s[36:37], v66, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v68, v18\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v68, v18\n"\
      "v_lshlrev_b64 v[48:49], 31, v[86:87]\n"\
      "v_lshlrev_b64 v[56:57], 7, v[90:91]\n"\
      "v_lshrrev_b64 v[32:33], 21, v[78:79]\n"\
      "v_lshrrev_b32 v52, 1, v87\n"\
      "v_lshrrev_b32 v60, 25, v91\n"\
      "v_lshrrev_b64 v[8:9], 9, v[94:95]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v69, v19, s[46:47]\n"\
      "v_lshlrev_b32 v36, 11, v78\n"\
      "v_lshlrev_b32 v12, 23, v94\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v69, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 27, v[74:75]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_lshrrev_b32 v28, 5, v75\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 15, v[82:83]\n"\
      "v_lshlrev_b64 v[16:17], 9, v[98:99]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_lshrrev_b32 v44, 17, v83\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v20, 23, v99\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v76, v34\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v77, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v76, v34\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v92, v10\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v73, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v77, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v93, v11, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v37, 1, v[32:33]\n"\
      "v_sub_co_u32_e64 v82, s[60:61], v80, v42\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v84, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[62:63], v81, v43, s[60:61]\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v84, v50\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v89, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 25, v[102:103]\n"\
      "v_lshlrev_b64 v[32:33], 1, v[106:107]\n"\
      "v_lshlrev_b64 v[8:9], 13, v[122:123]\n"\
      "v_lshrrev_b32 v28, 7, v103\n"\
      "v_lshrrev_b32 v36, 31, v107\n"\
      "v_lshrrev_b32 v12, 19, v123\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v85, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v82, s[60:61], v82, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v85, v51, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v44, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshrrev_b64 v[40:41], 15, v[110:111]\n"\
      "v_lshrrev_b64 v[56:57], 27, v[118:119]\n"\
      "v_lshrrev_b64 v[16:17], 3, v[126:127]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshlrev_b32 v44, 17, v110\n"\
      "v_lshlrev_b32 v60, 5, v118\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_lshlrev_b32 v20, 29, v126\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshlrev_b64 v[48:49], 21, v[114:115]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v52, 11, v115\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v108, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v116, v58\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v124, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v100, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v100, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_sub_co_u32_e64 v106, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v109, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v108, s[60:61], v108, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v114, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v117, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v116, s[72:73], v116, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_sub_co_u32_e64 v122, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v125, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v124, s[42:43], v124, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v101, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v101, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v107, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v109, s[62:63], v109, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v115, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v117, s[74:75], v117, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v123, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v125, s[44:45], v125, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v106, s[54:55], v106, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v108, s[60:61], v108, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v114, s[66:67], v114, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v116, s[72:73], v116, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v122, s[36:37], v122, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v124, s[42:43], v124, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "global_store_dwordx2 %[l8], v[64:65], s[78:79] offset:0\n"\
      "global_store_dwordx2 %[l8], v[66:67], s[78:79] offset:512\n"\
      "global_store_dwordx2 %[l8], v[68:69], s[78:79] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[70:71], s[78:79] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[72:73], s[78:79] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[74:75], s[78:79] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[76:77], s[78:79] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[78:79], s[78:79] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[80:81], s[80:81] offset:0\n"\
      "global_store_dwordx2 %[l8], v[82:83], s[80:81] offset:512\n"\
      "global_store_dwordx2 %[l8], v[84:85], s[80:81] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[86:87], s[80:81] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[88:89], s[80:81] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[90:91], s[80:81] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[92:93], s[80:81] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[94:95], s[80:81] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[96:97], s[82:83] offset:0\n"\
      "global_store_dwordx2 %[l8], v[98:99], s[82:83] offset:512\n"\
      "global_store_dwordx2 %[l8], v[100:101], s[82:83] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[102:103], s[82:83] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[104:105], s[82:83] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[106:107], s[82:83] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[108:109], s[82:83] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[110:111], s[82:83] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[112:113], s[84:85] offset:0\n"\
      "global_store_dwordx2 %[l8], v[114:115], s[84:85] offset:512\n"\
      "global_store_dwordx2 %[l8], v[116:117], s[84:85] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[118:119], s[84:85] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[120:121], s[84:85] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[122:123], s[84:85] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[124:125], s[84:85] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[126:127], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      :: __VA_ARGS__ \
      : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "scc", "memory")

// fwd_twist: 2001 VALU, 2211 lines
#define MI_TW_BODY_FWD_TWIST(...) asm volatile(\
      "s_mov_b64 s[22:23], exec\n"\
      "s_add_u32 s78, %[g_lo], 0\n"\
      "s_addc_u32 s79, %[g_hi], 0\n"\
      "s_add_u32 s80, %[g_lo], 4096\n"\
      "s_addc_u32 s81, %[g_hi], 0\n"\
      "s_add_u32 s82, %[g_lo], 8192\n"\
      "s_addc_u32 s83, %[g_hi], 0\n"\
      "s_add_u32 s84, %[g_lo], 12288\n"\
      "s_addc_u32 s85, %[g_hi], 0\n"\
      "s_add_u32 s86, %[tw_lo], 0\n"\
      "s_addc_u32 s87, %[tw_hi], 0\n"\
      "s_add_u32 s88, %[tw_lo], 4096\n"\
      "s_addc_u32 s89, %[tw_hi], 0\n"\
      "s_add_u32 s90, %[tw_lo], 8192\n"\
      "s_addc_u32 s91, %[tw_hi], 0\n"\
      "s_add_u32 s92, %[tw_lo], 12288\n"\
      "s_addc_u32 s93, %[tw_hi], 0\n"\
      "s_mov_b32 s20, 0xaaaaaaaa\n"\
      "s_mov_b32 s21, 0xaaaaaaaa\n"\
      "global_load_dwordx2 v[64:65], %[l8], s[78:79] offset:0\n"\
      "global_load_dwordx2 v[66:67], %[l8], s[78:79] offset:512\n"\
      "global_load_dwordx2 v[68:69], %[l8], s[78:79] offset:1024\n"\
      "global_load_dwordx2 v[70:71], %[l8], s[78:79] offset:1536\n"\
      "global_load_dwordx2 v[72:73], %[l8], s[78:79] offset:2048\n"\
      "global_load_dwordx2 v[74:75], %[l8], s[78:79] offset:2560\n"\
      "global_load_dwordx2 v[76:77], %[l8], s[78:79] offset:3072\n"\
      "global_load_dwordx2 v[78:79], %[l8], s[78:79] offset:3584\n"\
      "global_load_dwordx2 v[80:81], %[l8], s[80:81] offset:0\n"\
      "global_load_dwordx2 v[82:83], %[l8], s[80:81] offset:512\n"\
      "global_load_dwordx2 v[84:85], %[l8], s[80:81] offset:1024\n"\
      "global_load_dwordx2 v[86:87], %[l8], s[80:81] offset:1536\n"\
      "global_load_dwordx2 v[88:89], %[l8], s[80:81] offset:2048\n"\
      "global_load_dwordx2 v[90:91], %[l8], s[80:81] offset:2560\n"\
      "global_load_dwordx2 v[92:93], %[l8], s[80:81] offset:3072\n"\
      "global_load_dwordx2 v[94:95], %[l8], s[80:81] offset:3584\n"\
      "global_load_dwordx2 v[96:97], %[l8], s[82:83] offset:0\n"\
      "global_load_dwordx2 v[98:99], %[l8], s[82:83] offset:512\n"\
      "global_load_dwordx2 v[100:101], %[l8], s[82:83] offset:1024\n"\
      "global_load_dwordx2 v[102:103], %[l8], s[82:83] offset:1536\n"\
      "global_load_dwordx2 v[104:105], %[l8], s[82:83] offset:2048\n"\
      "global_load_dwordx2 v[106:107], %[l8], s[82:83] offset:2560\n"\
      "global_load_dwordx2 v[108:109], %[l8], s[82:83] offset:3072\n"\
      "global_load_dwordx2 v[110:111], %[l8], s[82:83] offset:3584\n"\
      "global_load_dwordx2 v[112:113], %[l8], s[84:85] offset:0\n"\
      "global_load_dwordx2 v[114:115], %[l8], s[84:85] offset:512\n"\
      "global_load_dwordx2 v[116:117], %[l8], s[84:85] offset:1024\n"\
      "global_load_dwordx2 v[118:119], %[l8], s[84:85] offset:1536\n"\
      "global_load_dwordx2 v[120:121], %[l8], s[84:85] offset:2048\n"\
      "global_load_dwordx2 v[122:123], %[l8], s[84:85] offset:2560\n"\
      "global_load_dwordx2 v[124:125], %[l8], s[84:85] offset:3072\n"\
      "global_load_dwordx2 v[126:127], %[l8], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_lshlrev_b64 v[8:9], 16, v[96:97]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[98:99]\n"\
      "v_lshrrev_b32 v12, 16, v97\n"\
      "v_lshrrev_b32 v20, 16, v99\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mov_b32 v14, 0\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v96, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v97, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v67, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v96, s[36:37], v96, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[100:101]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[102:103]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[104:105]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[106:107]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[108:109]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[110:111]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[112:113]\n"\
      "v_lshrrev_b32 v28, 16, v101\n"\
      "v_lshrrev_b32 v36, 16, v103\n"\
      "v_lshrrev_b32 v44, 16, v105\n"\
      "v_lshrrev_b32 v52, 16, v107\n"\
      "v_lshrrev_b32 v60, 16, v109\n"\
      "v_lshrrev_b32 v12, 16, v111\n"\
      "v_lshrrev_b32 v20, 16, v113\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v80, v18\n"\
      "v_sub_co_u32_e64 v100, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v102, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v104, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v106, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v108, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v110, s[36:37], v78, v10\n"\
      "v_sub_co_u32_e64 v112, s[42:43], v80, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v81, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v101, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v103, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v105, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v107, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v109, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v111, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v113, s[44:45], v81, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v100, s[48:49], v100, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v102, s[54:55], v102, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v104, s[60:61], v104, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v106, s[66:67], v106, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v108, s[72:73], v108, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v110, s[36:37], v110, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v112, s[42:43], v112, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[114:115]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[116:117]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[118:119]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[120:121]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[122:123]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[124:125]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[126:127]\n"\
      "v_lshrrev_b32 v28, 16, v115\n"\
      "v_lshrrev_b32 v36, 16, v117\n"\
      "v_lshrrev_b32 v44, 16, v119\n"\
      "v_lshrrev_b32 v52, 16, v121\n"\
      "v_lshrrev_b32 v60, 16, v123\n"\
      "v_lshrrev_b32 v12, 16, v125\n"\
      "v_lshrrev_b32 v20, 16, v127\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v82, v26\n"\
      "v_sub_co_u32_e64 v114, s[48:49], v82, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v84, v34\n"\
      "v_sub_co_u32_e64 v116, s[54:55], v84, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v86, v42\n"\
      "v_sub_co_u32_e64 v118, s[60:61], v86, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v88, v50\n"\
      "v_sub_co_u32_e64 v120, s[66:67], v88, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v90, v58\n"\
      "v_sub_co_u32_e64 v122, s[72:73], v90, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_sub_co_u32_e64 v124, s[36:37], v92, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v94, v18\n"\
      "v_sub_co_u32_e64 v126, s[42:43], v94, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v83, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v115, s[50:51], v83, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v85, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v117, s[56:57], v85, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v87, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v119, s[62:63], v87, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v89, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v121, s[68:69], v89, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v91, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v123, s[74:75], v91, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v125, s[38:39], v93, v11, s[36:37]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v95, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v127, s[44:45], v95, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v114, s[48:49], v114, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v116, s[54:55], v116, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v118, s[60:61], v118, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v120, s[66:67], v120, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v122, s[72:73], v122, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v124, s[36:37], v124, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v126, s[42:43], v126, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v127, s[24:25], v127, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[80:81]\n"\
      "v_lshlrev_b64 v[16:17], 24, v[82:83]\n"\
      "v_lshrrev_b32 v12, 8, v81\n"\
      "v_lshrrev_b32 v20, 8, v83\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v82, s[42:43], v66, v18\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v80, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[44:45], v67, v19, s[42:43]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v82, s[42:43], v82, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v80, s[36:37], v80, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v12, s[36:37]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[112:113]\n"\
      "v_lshlrev_b32 v20, 8, v112\n"\
      "v_lshlrev_b64 v[24:25], 24, v[84:85]\n"\
      "v_lshlrev_b64 v[32:33], 24, v[86:87]\n"\
      "v_lshlrev_b64 v[40:41], 24, v[88:89]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[94:95]\n"\
      "v_lshrrev_b32 v28, 8, v85\n"\
      "v_lshrrev_b32 v36, 8, v87\n"\
      "v_lshrrev_b32 v44, 8, v89\n"\
      "v_lshrrev_b32 v52, 8, v91\n"\
      "v_lshrrev_b32 v60, 8, v93\n"\
      "v_lshrrev_b32 v12, 8, v95\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_sub_co_u32_e64 v84, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v86, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v78, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v96, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v85, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v87, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v97, s[44:45], v97, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v84, s[48:49], v84, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v86, s[54:55], v86, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v96, s[42:43], v96, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v20, s[42:43]\n"\
      "v_lshrrev_b64 v[24:25], 24, v[114:115]\n"\
      "v_lshrrev_b64 v[32:33], 24, v[116:117]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[118:119]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 24, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 24, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[126:127]\n"\
      "v_lshlrev_b32 v28, 8, v114\n"\
      "v_lshlrev_b32 v36, 8, v116\n"\
      "v_lshlrev_b32 v44, 8, v118\n"\
      "v_lshlrev_b32 v52, 8, v120\n"\
      "v_lshlrev_b32 v60, 8, v122\n"\
      "v_lshlrev_b32 v12, 8, v124\n"\
      "v_lshlrev_b32 v20, 8, v126\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v28, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_sub_co_u32_e64 v27, s[48:49], v27, v28\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[48:49]\n"\
      "v_addc_co_u32_e64 v26, s[50:51], v26, 0, s[48:49]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v29, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v104, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v106, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v108, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v110, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_sub_co_u32_e64 v98, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v100, s[54:55], v100, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v102, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v105, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v104, s[66:67], v104, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v107, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v106, s[72:73], v106, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v109, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v108, s[36:37], v108, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v111, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v110, s[42:43], v110, v18\n"\
      "v_subb_co_u32_e64 v99, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v101, s[56:57], v101, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v103, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v105, s[68:69], v105, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v107, s[74:75], v107, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v109, s[38:39], v109, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v111, s[44:45], v111, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v98, s[48:49], v98, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v100, s[54:55], v100, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v102, s[60:61], v102, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v104, s[66:67], v104, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v106, s[72:73], v106, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v108, s[36:37], v108, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v110, s[42:43], v110, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[116:117], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 12, v[72:73]\n"\
      "v_lshlrev_b64 v[16:17], 12, v[74:75]\n"\
      "v_lshrrev_b32 v12, 20, v73\n"\
      "v_lshrrev_b32 v20, 20, v75\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v72, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v74, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v73, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v75, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 28, v[88:89]\n"\
      "v_lshrrev_b32 v44, 4, v89\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v72, s[36:37], v72, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v74, s[42:43], v74, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshlrev_b64 v[48:49], 28, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 28, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 28, v[94:95]\n"\
      "v_lshlrev_b64 v[16:17], 4, v[104:105]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshrrev_b32 v52, 4, v91\n"\
      "v_lshrrev_b32 v60, 4, v93\n"\
      "v_lshrrev_b32 v12, 4, v95\n"\
      "v_lshrrev_b32 v20, 28, v105\n"\
      "v_lshlrev_b64 v[24:25], 12, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 12, v[78:79]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 20, v77\n"\
      "v_lshrrev_b32 v36, 20, v79\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v81, v43, s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v84, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v86, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v82, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v84, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v86, v10\n"\
      "v_sub_co_u32_e64 v104, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v85, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v87, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v85, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v87, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v105, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 4, v[106:107]\n"\
      "v_lshlrev_b64 v[32:33], 4, v[108:109]\n"\
      "v_lshlrev_b64 v[40:41], 4, v[110:111]\n"\
      "v_lshrrev_b32 v28, 28, v107\n"\
      "v_lshrrev_b32 v36, 28, v109\n"\
      "v_lshrrev_b32 v44, 28, v111\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v104, s[42:43], v104, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 12, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 12, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 12, v[126:127]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 20, v120\n"\
      "v_lshlrev_b32 v60, 20, v122\n"\
      "v_lshlrev_b32 v12, 20, v124\n"\
      "v_lshlrev_b32 v20, 20, v126\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v116, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v118, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v106, s[48:49], v98, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_sub_co_u32_e64 v108, s[54:55], v100, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_sub_co_u32_e64 v110, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v112, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v114, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v117, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v116, s[36:37], v116, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v119, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v118, s[42:43], v118, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v107, s[50:51], v99, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v109, s[56:57], v101, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v111, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v113, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v115, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v117, s[38:39], v117, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v119, s[44:45], v119, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v106, s[48:49], v106, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v108, s[54:55], v108, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v110, s[60:61], v110, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v112, s[66:67], v112, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v114, s[72:73], v114, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v116, s[36:37], v116, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v118, s[42:43], v118, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 6, v[68:69]\n"\
      "v_lshrrev_b32 v12, 26, v69\n"\
      "v_lshlrev_b64 v[16:17], 6, v[70:71]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 26, v71\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_lshlrev_b64 v[24:25], 22, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 22, v[78:79]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshrrev_b32 v28, 10, v77\n"\
      "v_lshrrev_b32 v36, 10, v79\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v68, s[36:37], v64, v10\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v66, v18\n"\
      "v_subb_co_u32_e64 v69, s[38:39], v65, v11, s[36:37]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshrrev_b64 v[56:57], 18, v[92:93]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_lshlrev_b32 v60, 14, v92\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 30, v[84:85]\n"\
      "v_lshlrev_b64 v[48:49], 30, v[86:87]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v68, s[36:37], v68, 0, s[38:39]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v44, 2, v85\n"\
      "v_lshrrev_b32 v52, 2, v87\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_lshrrev_b64 v[8:9], 18, v[94:95]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_lshlrev_b32 v12, 14, v94\n"\
      "v_lshlrev_b64 v[16:17], 18, v[100:101]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 14, v101\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v82, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v88, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v89, s[74:75], v89, v59, s[72:73]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v90, v10\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v88, s[72:73], v88, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v74, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v74, v34\n"\
      "v_sub_co_u32_e64 v84, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v91, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v90, v10\n"\
      "v_sub_co_u32_e64 v100, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v60, s[72:73]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v75, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v72, v26\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v75, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v85, s[62:63], v81, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v91, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v101, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 10, v[116:117]\n"\
      "v_lshlrev_b64 v[56:57], 10, v[118:119]\n"\
      "v_lshrrev_b32 v52, 22, v117\n"\
      "v_lshrrev_b32 v60, 22, v119\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v73, v27, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v84, s[60:61], v84, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v100, s[42:43], v100, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_lshrrev_b64 v[32:33], 30, v[108:109]\n"\
      "v_lshrrev_b64 v[40:41], 30, v[110:111]\n"\
      "v_lshrrev_b64 v[8:9], 6, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 6, v[126:127]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_lshlrev_b32 v36, 2, v108\n"\
      "v_lshlrev_b32 v44, 2, v110\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v12, 26, v124\n"\
      "v_lshlrev_b32 v20, 26, v126\n"\
      "v_lshlrev_b64 v[24:25], 18, v[102:103]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 14, v103\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v106, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v122, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v104, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v107, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v106, s[60:61], v106, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v116, s[66:67], v112, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_sub_co_u32_e64 v118, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v120, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v123, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v122, s[42:43], v122, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v105, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v107, s[62:63], v107, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v117, s[68:69], v113, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v119, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v121, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v123, s[44:45], v123, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v104, s[54:55], v104, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v106, s[60:61], v106, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v116, s[66:67], v116, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v118, s[72:73], v118, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v120, s[36:37], v120, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v122, s[42:43], v122, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[16:17], 19, v[70:71]\n"\
      "v_lshlrev_b64 v[8:9], 3, v[66:67]\n"\
      "v_lshrrev_b32 v20, 13, v71\n"\
      "v_lshrrev_b32 v12, 29, v67\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_sub_co_u32_e64 v66, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_subb_co_u32_e64 v67, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v66, s[36:37], v66, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v68, v18\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v68, v18\n"\
      "v_lshlrev_b64 v[48:49], 31, v[86:87]\n"\
      "v_lshlrev_b64 v[56:57], 7, v[90:91]\n"\
      "v_lshrrev_b64 v[32:33], 21, v[78:79]\n"\
      "v_lshrrev_b32 v52, 1, v87\n"\
      "v_lshrrev_b32 v60, 25, v91\n"\
      "v_lshrrev_b64 v[8:9], 9, v[94:95]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v69, v19, s[46:47]\n"\
      "v_lshlrev_b32 v36, 11, v78\n"\
      "v_lshlrev_b32 v12, 23, v94\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v69, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 27, v[74:75]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_lshrrev_b32 v28, 5, v75\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 15, v[82:83]\n"\
      "v_lshlrev_b64 v[16:17], 9, v[98:99]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_lshrrev_b32 v44, 17, v83\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v20, 23, v99\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v76, v34\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v77, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v76, v34\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v92, v10\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v73, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v77, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v93, v11, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v37, 1, v[32:33]\n"\
      "v_sub_co_u32_e64 v82, s[60:61], v80, v42\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v84, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[62:63], v81, v43, s[60:61]\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v84, v50\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v89, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 25, v[102:103]\n"\
      "v_lshlrev_b64 v[32:33], 1, v[106:107]\n"\
      "v_lshlrev_b64 v[8:9], 13, v[122:123]\n"\
      "v_lshrrev_b32 v28, 7, v103\n"\
      "v_lshrrev_b32 v36, 31, v107\n"\
      "v_lshrrev_b32 v12, 19, v123\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v85, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v82, s[60:61], v82, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v85, v51, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v44, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshrrev_b64 v[40:41], 15, v[110:111]\n"\
      "v_lshrrev_b64 v[56:57], 27, v[118:119]\n"\
      "v_lshrrev_b64 v[16:17], 3, v[126:127]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshlrev_b32 v44, 17, v110\n"\
      "v_lshlrev_b32 v60, 5, v118\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_lshlrev_b32 v20, 29, v126\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshlrev_b64 v[48:49], 21, v[114:115]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v52, 11, v115\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v108, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v116, v58\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v124, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v100, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v100, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_sub_co_u32_e64 v106, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v109, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v108, s[60:61], v108, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v114, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v117, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v116, s[72:73], v116, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_sub_co_u32_e64 v122, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v125, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v124, s[42:43], v124, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v101, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v101, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v107, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v109, s[62:63], v109, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v115, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v117, s[74:75], v117, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v123, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v125, s[44:45], v125, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v106, s[54:55], v106, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v108, s[60:61], v108, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v114, s[66:67], v114, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v116, s[72:73], v116, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v122, s[36:37], v122, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v124, s[42:43], v124, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[86:87] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[86:87] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[86:87] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[86:87] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[86:87] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[86:87] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[86:87] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[86:87] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v64, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v66, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v64, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v66, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v65, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v65, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v67, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v67, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v68, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v64, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v65, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v66, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v67, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v70, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v72, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v68, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v70, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v72, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v69, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v69, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v71, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v71, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v73, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v73, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v68, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v69, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v70, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v71, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v72, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v73, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v74, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v76, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v78, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v74, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v76, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v78, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v75, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v75, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v77, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v77, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v79, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v79, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v74, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v75, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v76, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v77, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v78, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v79, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[88:89] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[88:89] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[88:89] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[88:89] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[88:89] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[88:89] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[88:89] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[88:89] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v80, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v82, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v80, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v82, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v81, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v81, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v83, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v83, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v84, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v80, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v81, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v82, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v83, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v86, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v88, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v84, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v86, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v88, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v85, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v85, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v87, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v87, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v89, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v89, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v84, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v85, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v86, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v87, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v88, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v89, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v90, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v92, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v94, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v90, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v92, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v94, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v91, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v91, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v93, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v93, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v95, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v95, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v90, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v91, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v92, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v93, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v94, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v95, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[90:91] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[90:91] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[90:91] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[90:91] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[90:91] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[90:91] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[90:91] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[90:91] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v96, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v98, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v96, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v98, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v97, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v97, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v99, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v99, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v100, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v96, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v97, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v98, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v99, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v102, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v104, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v100, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v102, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v104, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v101, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v101, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v103, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v103, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v105, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v105, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v100, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v101, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v102, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v103, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v104, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v106, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v108, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v110, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v106, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v108, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v110, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v107, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v107, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v109, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v109, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v111, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v111, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v106, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v107, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v108, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v109, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v110, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v111, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[92:93] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[92:93] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[92:93] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[92:93] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[92:93] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[92:93] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[92:93] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[92:93] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v112, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v114, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v112, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v114, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v113, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v113, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v115, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v115, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v116, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v112, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v113, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v114, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v115, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v118, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v120, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v116, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v118, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v120, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v117, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v117, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v119, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v119, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v121, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v121, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v116, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v117, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v118, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v119, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v120, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v121, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v122, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v124, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v126, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v122, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v124, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v126, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v123, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v123, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v125, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v125, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v127, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v127, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v122, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v123, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v124, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v125, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v126, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v127, v37, v41, s[44:45]\n"\
      "global_store_dwordx2 %[l8], v[64:65], s[78:79] offset:0\n"\
      "global_store_dwordx2 %[l8], v[66:67], s[78:79] offset:512\n"\
      "global_store_dwordx2 %[l8], v[68:69], s[78:79] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[70:71], s[78:79] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[72:73], s[78:79] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[74:75], s[78:79] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[76:77], s[78:79] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[78:79], s[78:79] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[80:81], s[80:81] offset:0\n"\
      "global_store_dwordx2 %[l8], v[82:83], s[80:81] offset:512\n"\
      "global_store_dwordx2 %[l8], v[84:85], s[80:81] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[86:87], s[80:81] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[88:89], s[80:81] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[90:91], s[80:81] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[92:93], s[80:81] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[94:95], s[80:81] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[96:97], s[82:83] offset:0\n"\
      "global_store_dwordx2 %[l8], v[98:99], s[82:83] offset:512\n"\
      "global_store_dwordx2 %[l8], v[100:101], s[82:83] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[102:103], s[82:83] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[104:105], s[82:83] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[106:107], s[82:83] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[108:109], s[82:83] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[110:111], s[82:83] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[112:113], s[84:85] offset:0\n"\
      "global_store_dwordx2 %[l8], v[114:115], s[84:85] offset:512\n"\
      "global_store_dwordx2 %[l8], v[116:117], s[84:85] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[118:119], s[84:85] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[120:121], s[84:85] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[122:123], s[84:85] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[124:125], s[84:85] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[126:127], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      :: __VA_ARGS__ \
      : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "scc", "memory")

// fwd_t1: 2001 VALU, 2315 lines
#define MI_TW_BODY_FWD_T1(...) asm volatile(\
      "s_mov_b64 s[22:23], exec\n"\
      "s_add_u32 s78, %[g_lo], 0\n"\
      "s_addc_u32 s79, %[g_hi], 0\n"\
      "s_add_u32 s80, %[g_lo], 4096\n"\
      "s_addc_u32 s81, %[g_hi], 0\n"\
      "s_add_u32 s82, %[g_lo], 8192\n"\
      "s_addc_u32 s83, %[g_hi], 0\n"\
      "s_add_u32 s84, %[g_lo], 12288\n"\
      "s_addc_u32 s85, %[g_hi], 0\n"\
      "s_add_u32 s86, %[tw_lo], 0\n"\
      "s_addc_u32 s87, %[tw_hi], 0\n"\
      "s_add_u32 s88, %[tw_lo], 4096\n"\
      "s_addc_u32 s89, %[tw_hi], 0\n"\
      "s_add_u32 s90, %[tw_lo], 8192\n"\
      "s_addc_u32 s91, %[tw_hi], 0\n"\
      "s_add_u32 s92, %[tw_lo], 12288\n"\
      "s_addc_u32 s93, %[tw_hi], 0\n"\
      "s_mov_b32 s20, 0xaaaaaaaa\n"\
      "s_mov_b32 s21, 0xaaaaaaaa\n"\
      "global_load_dwordx2 v[64:65], %[l8], s[78:79] offset:0\n"\
      "global_load_dwordx2 v[66:67], %[l8], s[78:79] offset:512\n"\
      "global_load_dwordx2 v[68:69], %[l8], s[78:79] offset:1024\n"\
      "global_load_dwordx2 v[70:71], %[l8], s[78:79] offset:1536\n"\
      "global_load_dwordx2 v[72:73], %[l8], s[78:79] offset:2048\n"\
      "global_load_dwordx2 v[74:75], %[l8], s[78:79] offset:2560\n"\
      "global_load_dwordx2 v[76:77], %[l8], s[78:79] offset:3072\n"\
      "global_load_dwordx2 v[78:79], %[l8], s[78:79] offset:3584\n"\
      "global_load_dwordx2 v[80:81], %[l8], s[80:81] offset:0\n"\
      "global_load_dwordx2 v[82:83], %[l8], s[80:81] offset:512\n"\
      "global_load_dwordx2 v[84:85], %[l8], s[80:81] offset:1024\n"\
      "global_load_dwordx2 v[86:87], %[l8], s[80:81] offset:1536\n"\
      "global_load_dwordx2 v[88:89], %[l8], s[80:81] offset:2048\n"\
      "global_load_dwordx2 v[90:91], %[l8], s[80:81] offset:2560\n"\
      "global_load_dwordx2 v[92:93], %[l8], s[80:81] offset:3072\n"\
      "global_load_dwordx2 v[94:95], %[l8], s[80:81] offset:3584\n"\
      "global_load_dwordx2 v[96:97], %[l8], s[82:83] offset:0\n"\
      "global_load_dwordx2 v[98:99], %[l8], s[82:83] offset:512\n"\
      "global_load_dwordx2 v[100:101], %[l8], s[82:83] offset:1024\n"\
      "global_load_dwordx2 v[102:103], %[l8], s[82:83] offset:1536\n"\
      "global_load_dwordx2 v[104:105], %[l8], s[82:83] offset:2048\n"\
      "global_load_dwordx2 v[106:107], %[l8], s[82:83] offset:2560\n"\
      "global_load_dwordx2 v[108:109], %[l8], s[82:83] offset:3072\n"\
      "global_load_dwordx2 v[110:111], %[l8], s[82:83] offset:3584\n"\
      "global_load_dwordx2 v[112:113], %[l8], s[84:85] offset:0\n"\
      "global_load_dwordx2 v[114:115], %[l8], s[84:85] offset:512\n"\
      "global_load_dwordx2 v[116:117], %[l8], s[84:85] offset:1024\n"\
      "global_load_dwordx2 v[118:119], %[l8], s[84:85] offset:1536\n"\
      "global_load_dwordx2 v[120:121], %[l8], s[84:85] offset:2048\n"\
      "global_load_dwordx2 v[122:123], %[l8], s[84:85] offset:2560\n"\
      "global_load_dwordx2 v[124:125], %[l8], s[84:85] offset:3072\n"\
      "global_load_dwordx2 v[126:127], %[l8], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_lshlrev_b64 v[8:9], 16, v[96:97]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[98:99]\n"\
      "v_lshrrev_b32 v12, 16, v97\n"\
      "v_lshrrev_b32 v20, 16, v99\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mov_b32 v14, 0\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v96, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v97, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v67, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v96, s[36:37], v96, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[100:101]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[102:103]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[104:105]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[106:107]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[108:109]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[110:111]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[112:113]\n"\
      "v_lshrrev_b32 v28, 16, v101\n"\
      "v_lshrrev_b32 v36, 16, v103\n"\
      "v_lshrrev_b32 v44, 16, v105\n"\
      "v_lshrrev_b32 v52, 16, v107\n"\
      "v_lshrrev_b32 v60, 16, v109\n"\
      "v_lshrrev_b32 v12, 16, v111\n"\
      "v_lshrrev_b32 v20, 16, v113\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v80, v18\n"\
      "v_sub_co_u32_e64 v100, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v102, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v104, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v106, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v108, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v110, s[36:37], v78, v10\n"\
      "v_sub_co_u32_e64 v112, s[42:43], v80, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v81, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v101, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v103, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v105, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v107, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v109, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v111, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v113, s[44:45], v81, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v100, s[48:49], v100, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v102, s[54:55], v102, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v104, s[60:61], v104, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v106, s[66:67], v106, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v108, s[72:73], v108, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v110, s[36:37], v110, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v112, s[42:43], v112, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[114:115]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[116:117]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[118:119]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[120:121]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[122:123]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[124:125]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[126:127]\n"\
      "v_lshrrev_b32 v28, 16, v115\n"\
      "v_lshrrev_b32 v36, 16, v117\n"\
      "v_lshrrev_b32 v44, 16, v119\n"\
      "v_lshrrev_b32 v52, 16, v121\n"\
      "v_lshrrev_b32 v60, 16, v123\n"\
      "v_lshrrev_b32 v12, 16, v125\n"\
      "v_lshrrev_b32 v20, 16, v127\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v82, v26\n"\
      "v_sub_co_u32_e64 v114, s[48:49], v82, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v84, v34\n"\
      "v_sub_co_u32_e64 v116, s[54:55], v84, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v86, v42\n"\
      "v_sub_co_u32_e64 v118, s[60:61], v86, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v88, v50\n"\
      "v_sub_co_u32_e64 v120, s[66:67], v88, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v90, v58\n"\
      "v_sub_co_u32_e64 v122, s[72:73], v90, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_sub_co_u32_e64 v124, s[36:37], v92, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v94, v18\n"\
      "v_sub_co_u32_e64 v126, s[42:43], v94, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v83, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v115, s[50:51], v83, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v85, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v117, s[56:57], v85, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v87, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v119, s[62:63], v87, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v89, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v121, s[68:69], v89, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v91, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v123, s[74:75], v91, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v125, s[38:39], v93, v11, s[36:37]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v95, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v127, s[44:45], v95, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v114, s[48:49], v114, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v116, s[54:55], v116, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v118, s[60:61], v118, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v120, s[66:67], v120, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v122, s[72:73], v122, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v124, s[36:37], v124, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v126, s[42:43], v126, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v127, s[24:25], v127, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[80:81]\n"\
      "v_lshlrev_b64 v[16:17], 24, v[82:83]\n"\
      "v_lshrrev_b32 v12, 8, v81\n"\
      "v_lshrrev_b32 v20, 8, v83\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v82, s[42:43], v66, v18\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v80, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[44:45], v67, v19, s[42:43]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v82, s[42:43], v82, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v80, s[36:37], v80, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v12, s[36:37]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[112:113]\n"\
      "v_lshlrev_b32 v20, 8, v112\n"\
      "v_lshlrev_b64 v[24:25], 24, v[84:85]\n"\
      "v_lshlrev_b64 v[32:33], 24, v[86:87]\n"\
      "v_lshlrev_b64 v[40:41], 24, v[88:89]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[94:95]\n"\
      "v_lshrrev_b32 v28, 8, v85\n"\
      "v_lshrrev_b32 v36, 8, v87\n"\
      "v_lshrrev_b32 v44, 8, v89\n"\
      "v_lshrrev_b32 v52, 8, v91\n"\
      "v_lshrrev_b32 v60, 8, v93\n"\
      "v_lshrrev_b32 v12, 8, v95\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_sub_co_u32_e64 v84, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v86, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v78, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v96, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v85, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v87, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v97, s[44:45], v97, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v84, s[48:49], v84, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v86, s[54:55], v86, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v96, s[42:43], v96, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v20, s[42:43]\n"\
      "v_lshrrev_b64 v[24:25], 24, v[114:115]\n"\
      "v_lshrrev_b64 v[32:33], 24, v[116:117]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[118:119]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 24, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 24, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[126:127]\n"\
      "v_lshlrev_b32 v28, 8, v114\n"\
      "v_lshlrev_b32 v36, 8, v116\n"\
      "v_lshlrev_b32 v44, 8, v118\n"\
      "v_lshlrev_b32 v52, 8, v120\n"\
      "v_lshlrev_b32 v60, 8, v122\n"\
      "v_lshlrev_b32 v12, 8, v124\n"\
      "v_lshlrev_b32 v20, 8, v126\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v28, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_sub_co_u32_e64 v27, s[48:49], v27, v28\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[48:49]\n"\
      "v_addc_co_u32_e64 v26, s[50:51], v26, 0, s[48:49]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v29, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v104, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v106, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v108, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v110, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_sub_co_u32_e64 v98, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v100, s[54:55], v100, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v102, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v105, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v104, s[66:67], v104, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v107, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v106, s[72:73], v106, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v109, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v108, s[36:37], v108, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v111, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v110, s[42:43], v110, v18\n"\
      "v_subb_co_u32_e64 v99, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v101, s[56:57], v101, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v103, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v105, s[68:69], v105, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v107, s[74:75], v107, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v109, s[38:39], v109, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v111, s[44:45], v111, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v98, s[48:49], v98, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v100, s[54:55], v100, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v102, s[60:61], v102, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v104, s[66:67], v104, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v106, s[72:73], v106, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v108, s[36:37], v108, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v110, s[42:43], v110, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[116:117], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 12, v[72:73]\n"\
      "v_lshlrev_b64 v[16:17], 12, v[74:75]\n"\
      "v_lshrrev_b32 v12, 20, v73\n"\
      "v_lshrrev_b32 v20, 20, v75\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v72, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v74, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v73, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v75, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 28, v[88:89]\n"\
      "v_lshrrev_b32 v44, 4, v89\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v72, s[36:37], v72, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v74, s[42:43], v74, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshlrev_b64 v[48:49], 28, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 28, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 28, v[94:95]\n"\
      "v_lshlrev_b64 v[16:17], 4, v[104:105]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshrrev_b32 v52, 4, v91\n"\
      "v_lshrrev_b32 v60, 4, v93\n"\
      "v_lshrrev_b32 v12, 4, v95\n"\
      "v_lshrrev_b32 v20, 28, v105\n"\
      "v_lshlrev_b64 v[24:25], 12, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 12, v[78:79]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 20, v77\n"\
      "v_lshrrev_b32 v36, 20, v79\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v81, v43, s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v84, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v86, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v82, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v84, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v86, v10\n"\
      "v_sub_co_u32_e64 v104, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v85, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v87, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v85, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v87, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v105, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 4, v[106:107]\n"\
      "v_lshlrev_b64 v[32:33], 4, v[108:109]\n"\
      "v_lshlrev_b64 v[40:41], 4, v[110:111]\n"\
      "v_lshrrev_b32 v28, 28, v107\n"\
      "v_lshrrev_b32 v36, 28, v109\n"\
      "v_lshrrev_b32 v44, 28, v111\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v104, s[42:43], v104, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 12, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 12, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 12, v[126:127]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 20, v120\n"\
      "v_lshlrev_b32 v60, 20, v122\n"\
      "v_lshlrev_b32 v12, 20, v124\n"\
      "v_lshlrev_b32 v20, 20, v126\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v116, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v118, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v106, s[48:49], v98, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_sub_co_u32_e64 v108, s[54:55], v100, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_sub_co_u32_e64 v110, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v112, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v114, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v117, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v116, s[36:37], v116, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v119, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v118, s[42:43], v118, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v107, s[50:51], v99, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v109, s[56:57], v101, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v111, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v113, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v115, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v117, s[38:39], v117, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v119, s[44:45], v119, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v106, s[48:49], v106, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v108, s[54:55], v108, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v110, s[60:61], v110, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v112, s[66:67], v112, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v114, s[72:73], v114, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v116, s[36:37], v116, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v118, s[42:43], v118, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 6, v[68:69]\n"\
      "v_lshrrev_b32 v12, 26, v69\n"\
      "v_lshlrev_b64 v[16:17], 6, v[70:71]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 26, v71\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_lshlrev_b64 v[24:25], 22, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 22, v[78:79]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshrrev_b32 v28, 10, v77\n"\
      "v_lshrrev_b32 v36, 10, v79\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v68, s[36:37], v64, v10\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v66, v18\n"\
      "v_subb_co_u32_e64 v69, s[38:39], v65, v11, s[36:37]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshrrev_b64 v[56:57], 18, v[92:93]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_lshlrev_b32 v60, 14, v92\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 30, v[84:85]\n"\
      "v_lshlrev_b64 v[48:49], 30, v[86:87]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v68, s[36:37], v68, 0, s[38:39]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v44, 2, v85\n"\
      "v_lshrrev_b32 v52, 2, v87\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_lshrrev_b64 v[8:9], 18, v[94:95]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_lshlrev_b32 v12, 14, v94\n"\
      "v_lshlrev_b64 v[16:17], 18, v[100:101]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 14, v101\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v82, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v88, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v89, s[74:75], v89, v59, s[72:73]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v90, v10\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v88, s[72:73], v88, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v74, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v74, v34\n"\
      "v_sub_co_u32_e64 v84, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v91, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v90, v10\n"\
      "v_sub_co_u32_e64 v100, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v60, s[72:73]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v75, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v72, v26\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v75, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v85, s[62:63], v81, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v91, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v101, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 10, v[116:117]\n"\
      "v_lshlrev_b64 v[56:57], 10, v[118:119]\n"\
      "v_lshrrev_b32 v52, 22, v117\n"\
      "v_lshrrev_b32 v60, 22, v119\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v73, v27, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v84, s[60:61], v84, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v100, s[42:43], v100, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_lshrrev_b64 v[32:33], 30, v[108:109]\n"\
      "v_lshrrev_b64 v[40:41], 30, v[110:111]\n"\
      "v_lshrrev_b64 v[8:9], 6, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 6, v[126:127]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_lshlrev_b32 v36, 2, v108\n"\
      "v_lshlrev_b32 v44, 2, v110\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v12, 26, v124\n"\
      "v_lshlrev_b32 v20, 26, v126\n"\
      "v_lshlrev_b64 v[24:25], 18, v[102:103]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 14, v103\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v106, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v122, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v104, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v107, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v106, s[60:61], v106, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v116, s[66:67], v112, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_sub_co_u32_e64 v118, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v120, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v123, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v122, s[42:43], v122, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v105, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v107, s[62:63], v107, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v117, s[68:69], v113, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v119, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v121, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v123, s[44:45], v123, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v104, s[54:55], v104, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v106, s[60:61], v106, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v116, s[66:67], v116, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v118, s[72:73], v118, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v120, s[36:37], v120, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v122, s[42:43], v122, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[16:17], 19, v[70:71]\n"\
      "v_lshlrev_b64 v[8:9], 3, v[66:67]\n"\
      "v_lshrrev_b32 v20, 13, v71\n"\
      "v_lshrrev_b32 v12, 29, v67\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_sub_co_u32_e64 v66, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_subb_co_u32_e64 v67, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v66, s[36:37], v66, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v68, v18\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v68, v18\n"\
      "v_lshlrev_b64 v[48:49], 31, v[86:87]\n"\
      "v_lshlrev_b64 v[56:57], 7, v[90:91]\n"\
      "v_lshrrev_b64 v[32:33], 21, v[78:79]\n"\
      "v_lshrrev_b32 v52, 1, v87\n"\
      "v_lshrrev_b32 v60, 25, v91\n"\
      "v_lshrrev_b64 v[8:9], 9, v[94:95]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v69, v19, s[46:47]\n"\
      "v_lshlrev_b32 v36, 11, v78\n"\
      "v_lshlrev_b32 v12, 23, v94\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v69, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 27, v[74:75]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_lshrrev_b32 v28, 5, v75\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 15, v[82:83]\n"\
      "v_lshlrev_b64 v[16:17], 9, v[98:99]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_lshrrev_b32 v44, 17, v83\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v20, 23, v99\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v76, v34\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v77, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v76, v34\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v92, v10\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v73, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v77, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v93, v11, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v37, 1, v[32:33]\n"\
      "v_sub_co_u32_e64 v82, s[60:61], v80, v42\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v84, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[62:63], v81, v43, s[60:61]\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v84, v50\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v89, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 25, v[102:103]\n"\
      "v_lshlrev_b64 v[32:33], 1, v[106:107]\n"\
      "v_lshlrev_b64 v[8:9], 13, v[122:123]\n"\
      "v_lshrrev_b32 v28, 7, v103\n"\
      "v_lshrrev_b32 v36, 31, v107\n"\
      "v_lshrrev_b32 v12, 19, v123\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v85, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v82, s[60:61], v82, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v85, v51, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v44, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshrrev_b64 v[40:41], 15, v[110:111]\n"\
      "v_lshrrev_b64 v[56:57], 27, v[118:119]\n"\
      "v_lshrrev_b64 v[16:17], 3, v[126:127]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshlrev_b32 v44, 17, v110\n"\
      "v_lshlrev_b32 v60, 5, v118\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_lshlrev_b32 v20, 29, v126\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshlrev_b64 v[48:49], 21, v[114:115]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v52, 11, v115\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v108, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v116, v58\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v124, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v100, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v100, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_sub_co_u32_e64 v106, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v109, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v108, s[60:61], v108, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v114, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v117, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v116, s[72:73], v116, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_sub_co_u32_e64 v122, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v125, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v124, s[42:43], v124, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v101, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v101, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v107, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v109, s[62:63], v109, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v115, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v117, s[74:75], v117, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v123, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v125, s[44:45], v125, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v106, s[54:55], v106, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v108, s[60:61], v108, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v114, s[66:67], v114, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v116, s[72:73], v116, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v122, s[36:37], v122, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v124, s[42:43], v124, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[86:87] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[86:87] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[86:87] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[86:87] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[86:87] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[86:87] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[86:87] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[86:87] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v64, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v66, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v64, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v66, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v65, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v65, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v67, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v67, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v68, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v64, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v65, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v66, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v67, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v70, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v72, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v68, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v70, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v72, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v69, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v69, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v71, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v71, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v73, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v73, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v68, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v69, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v70, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v71, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v72, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v73, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v74, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v76, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v78, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v74, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v76, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v78, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v75, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v75, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v77, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v77, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v79, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v79, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v74, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v75, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v76, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v77, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v78, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v79, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[88:89] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[88:89] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[88:89] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[88:89] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[88:89] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[88:89] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[88:89] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[88:89] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v80, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v82, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v80, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v82, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v81, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v81, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v83, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v83, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v84, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v80, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v81, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v82, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v83, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v86, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v88, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v84, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v86, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v88, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v85, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v85, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v87, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v87, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v89, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v89, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v84, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v85, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v86, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v87, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v88, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v89, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v90, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v92, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v94, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v90, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v92, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v94, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v91, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v91, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v93, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v93, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v95, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v95, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v90, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v91, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v92, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v93, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v94, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v95, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[90:91] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[90:91] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[90:91] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[90:91] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[90:91] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[90:91] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[90:91] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[90:91] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v96, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v98, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v96, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v98, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v97, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v97, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v99, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v99, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v100, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v96, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v97, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v98, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v99, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v102, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v104, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v100, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v102, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v104, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v101, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v101, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v103, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v103, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v105, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v105, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v100, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v101, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v102, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v103, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v104, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v106, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v108, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v110, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v106, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v108, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v110, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v107, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v107, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v109, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v109, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v111, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v111, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v106, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v107, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v108, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v109, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v110, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v111, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[92:93] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[92:93] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[92:93] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[92:93] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[92:93] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[92:93] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[92:93] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[92:93] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v112, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v114, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v112, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v114, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v113, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v113, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v115, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v115, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v116, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v112, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v113, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v114, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v115, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v118, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v120, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v116, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v118, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v120, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v117, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v117, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v119, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v119, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v121, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v121, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v116, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v117, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v118, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v119, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v120, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v121, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v122, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v124, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v126, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v122, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v124, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v126, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v123, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v123, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v125, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v125, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v127, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v127, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v122, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v123, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v124, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v125, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v126, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v127, v37, v41, s[44:45]\n"\
      "s_mov_b32 exec_lo, -1\n"\
      "s_mov_b32 exec_hi, 0\n"\
      "ds_write_b64 %[t1w], v[64:65] offset:0\n"\
      "ds_write_b64 %[t1w], v[66:67] offset:272\n"\
      "ds_write_b64 %[t1w], v[68:69] offset:544\n"\
      "ds_write_b64 %[t1w], v[70:71] offset:816\n"\
      "ds_write_b64 %[t1w], v[72:73] offset:1088\n"\
      "ds_write_b64 %[t1w], v[74:75] offset:1360\n"\
      "ds_write_b64 %[t1w], v[76:77] offset:1632\n"\
      "ds_write_b64 %[t1w], v[78:79] offset:1904\n"\
      "ds_write_b64 %[t1w], v[80:81] offset:2176\n"\
      "ds_write_b64 %[t1w], v[82:83] offset:2448\n"\
      "ds_write_b64 %[t1w], v[84:85] offset:2720\n"\
      "ds_write_b64 %[t1w], v[86:87] offset:2992\n"\
      "ds_write_b64 %[t1w], v[88:89] offset:3264\n"\
      "ds_write_b64 %[t1w], v[90:91] offset:3536\n"\
      "ds_write_b64 %[t1w], v[92:93] offset:3808\n"\
      "ds_write_b64 %[t1w], v[94:95] offset:4080\n"\
      "ds_write_b64 %[t1w], v[96:97] offset:4352\n"\
      "ds_write_b64 %[t1w], v[98:99] offset:4624\n"\
      "ds_write_b64 %[t1w], v[100:101] offset:4896\n"\
      "ds_write_b64 %[t1w], v[102:103] offset:5168\n"\
      "ds_write_b64 %[t1w], v[104:105] offset:5440\n"\
      "ds_write_b64 %[t1w], v[106:107] offset:5712\n"\
      "ds_write_b64 %[t1w], v[108:109] offset:5984\n"\
      "ds_write_b64 %[t1w], v[110:111] offset:6256\n"\
      "ds_write_b64 %[t1w], v[112:113] offset:6528\n"\
      "ds_write_b64 %[t1w], v[114:115] offset:6800\n"\
      "ds_write_b64 %[t1w], v[116:117] offset:7072\n"\
      "ds_write_b64 %[t1w], v[118:119] offset:7344\n"\
      "ds_write_b64 %[t1w], v[120:121] offset:7616\n"\
      "ds_write_b64 %[t1w], v[122:123] offset:7888\n"\
      "ds_write_b64 %[t1w], v[124:125] offset:8160\n"\
      "ds_write_b64 %[t1w], v[126:127] offset:8432\n"\
      "s_mov_b64 exec, s[22:23]\n"\
      "ds_read_b64 v[8:9], %[t1r] offset:0\n"\
      "ds_read_b64 v[10:11], %[t1r] offset:16\n"\
      "ds_read_b64 v[12:13], %[t1r] offset:32\n"\
      "ds_read_b64 v[14:15], %[t1r] offset:48\n"\
      "ds_read_b64 v[16:17], %[t1r] offset:64\n"\
      "ds_read_b64 v[18:19], %[t1r] offset:80\n"\
      "ds_read_b64 v[20:21], %[t1r] offset:96\n"\
      "ds_read_b64 v[22:23], %[t1r] offset:112\n"\
      "ds_read_b64 v[24:25], %[t1r] offset:128\n"\
      "ds_read_b64 v[26:27], %[t1r] offset:144\n"\
      "ds_read_b64 v[28:29], %[t1r] offset:160\n"\
      "ds_read_b64 v[30:31], %[t1r] offset:176\n"\
      "ds_read_b64 v[32:33], %[t1r] offset:192\n"\
      "ds_read_b64 v[34:35], %[t1r] offset:208\n"\
      "ds_read_b64 v[36:37], %[t1r] offset:224\n"\
      "ds_read_b64 v[38:39], %[t1r] offset:240\n"\
      "s_mov_b32 exec_lo, 0\n"\
      "s_mov_b32 exec_hi, -1\n"\
      "ds_write_b64 %[t1w], v[64:65] offset:0\n"\
      "ds_write_b64 %[t1w], v[66:67] offset:272\n"\
      "ds_write_b64 %[t1w], v[68:69] offset:544\n"\
      "ds_write_b64 %[t1w], v[70:71] offset:816\n"\
      "ds_write_b64 %[t1w], v[72:73] offset:1088\n"\
      "ds_write_b64 %[t1w], v[74:75] offset:1360\n"\
      "ds_write_b64 %[t1w], v[76:77] offset:1632\n"\
      "ds_write_b64 %[t1w], v[78:79] offset:1904\n"\
      "ds_write_b64 %[t1w], v[80:81] offset:2176\n"\
      "ds_write_b64 %[t1w], v[82:83] offset:2448\n"\
      "ds_write_b64 %[t1w], v[84:85] offset:2720\n"\
      "ds_write_b64 %[t1w], v[86:87] offset:2992\n"\
      "ds_write_b64 %[t1w], v[88:89] offset:3264\n"\
      "ds_write_b64 %[t1w], v[90:91] offset:3536\n"\
      "ds_write_b64 %[t1w], v[92:93] offset:3808\n"\
      "ds_write_b64 %[t1w], v[94:95] offset:4080\n"\
      "ds_write_b64 %[t1w], v[96:97] offset:4352\n"\
      "ds_write_b64 %[t1w], v[98:99] offset:4624\n"\
      "ds_write_b64 %[t1w], v[100:101] offset:4896\n"\
      "ds_write_b64 %[t1w], v[102:103] offset:5168\n"\
      "ds_write_b64 %[t1w], v[104:105] offset:5440\n"\
      "ds_write_b64 %[t1w], v[106:107] offset:5712\n"\
      "ds_write_b64 %[t1w], v[108:109] offset:5984\n"\
      "ds_write_b64 %[t1w], v[110:111] offset:6256\n"\
      "ds_write_b64 %[t1w], v[112:113] offset:6528\n"\
      "ds_write_b64 %[t1w], v[114:115] offset:6800\n"\
      "ds_write_b64 %[t1w], v[116:117] offset:7072\n"\
      "ds_write_b64 %[t1w], v[118:119] offset:7344\n"\
      "ds_write_b64 %[t1w], v[120:121] offset:7616\n"\
      "ds_write_b64 %[t1w], v[122:123] offset:7888\n"\
      "ds_write_b64 %[t1w], v[124:125] offset:8160\n"\
      "ds_write_b64 %[t1w], v[126:127] offset:8432\n"\
      "s_mov_b64 exec, s[22:23]\n"\
      "s_waitcnt lgkmcnt(0)\n"\
      "ds_read_b64 v[64:65], %[t1r] offset:0\n"\
      "ds_read_b64 v[66:67], %[t1r] offset:16\n"\
      "ds_read_b64 v[68:69], %[t1r] offset:32\n"\
      "ds_read_b64 v[70:71], %[t1r] offset:48\n"\
      "ds_read_b64 v[72:73], %[t1r] offset:64\n"\
      "ds_read_b64 v[74:75], %[t1r] offset:80\n"\
      "ds_read_b64 v[76:77], %[t1r] offset:96\n"\
      "ds_read_b64 v[78:79], %[t1r] offset:112\n"\
      "ds_read_b64 v[80:81], %[t1r] offset:128\n"\
      "ds_read_b64 v[82:83], %[t1r] offset:144\n"\
      "ds_read_b64 v[84:85], %[t1r] offset:160\n"\
      "ds_read_b64 v[86:87], %[t1r] offset:176\n"\
      "ds_read_b64 v[88:89], %[t1r] offset:192\n"\
      "ds_read_b64 v[90:91], %[t1r] offset:208\n"\
      "ds_read_b64 v[92:93], %[t1r] offset:224\n"\
      "ds_read_b64 v[94:95], %[t1r] offset:240\n"\
      "s_waitcnt lgkmcnt(0)\n"\
      "global_store_dwordx2 %[l8], v[8:9], s[78:79] offset:0\n"\
      "global_store_dwordx2 %[l8], v[10:11], s[78:79] offset:512\n"\
      "global_store_dwordx2 %[l8], v[12:13], s[78:79] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[14:15], s[78:79] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[16:17], s[78:79] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[18:19], s[78:79] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[20:21], s[78:79] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[22:23], s[78:79] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[24:25], s[80:81] offset:0\n"\
      "global_store_dwordx2 %[l8], v[26:27], s[80:81] offset:512\n"\
      "global_store_dwordx2 %[l8], v[28:29], s[80:81] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[30:31], s[80:81] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[32:33], s[80:81] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[34:35], s[80:81] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[36:37], s[80:81] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[38:39], s[80:81] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[64:65], s[82:83] offset:0\n"\
      "global_store_dwordx2 %[l8], v[66:67], s[82:83] offset:512\n"\
      "global_store_dwordx2 %[l8], v[68:69], s[82:83] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[70:71], s[82:83] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[72:73], s[82:83] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[74:75], s[82:83] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[76:77], s[82:83] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[78:79], s[82:83] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[80:81], s[84:85] offset:0\n"\
      "global_store_dwordx2 %[l8], v[82:83], s[84:85] offset:512\n"\
      "global_store_dwordx2 %[l8], v[84:85], s[84:85] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[86:87], s[84:85] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[88:89], s[84:85] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[90:91], s[84:85] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[92:93], s[84:85] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[94:95], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      :: __VA_ARGS__ \
      : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "scc", "memory")

// fwd_cyc: 3236 VALU, 3586 lines
#define MI_TW_BODY_FWD_CYC(...) asm volatile(\
      "s_mov_b64 s[22:23], exec\n"\
      "s_add_u32 s78, %[g_lo], 0\n"\
      "s_addc_u32 s79, %[g_hi], 0\n"\
      "s_add_u32 s80, %[g_lo], 4096\n"\
      "s_addc_u32 s81, %[g_hi], 0\n"\
      "s_add_u32 s82, %[g_lo], 8192\n"\
      "s_addc_u32 s83, %[g_hi], 0\n"\
      "s_add_u32 s84, %[g_lo], 12288\n"\
      "s_addc_u32 s85, %[g_hi], 0\n"\
      "s_add_u32 s86, %[tw_lo], 0\n"\
      "s_addc_u32 s87, %[tw_hi], 0\n"\
      "s_add_u32 s88, %[tw_lo], 4096\n"\
      "s_addc_u32 s89, %[tw_hi], 0\n"\
      "s_add_u32 s90, %[tw_lo], 8192\n"\
      "s_addc_u32 s91, %[tw_hi], 0\n"\
      "s_add_u32 s92, %[tw_lo], 12288\n"\
      "s_addc_u32 s93, %[tw_hi], 0\n"\
      "s_mov_b32 s20, 0xaaaaaaaa\n"\
      "s_mov_b32 s21, 0xaaaaaaaa\n"\
      "global_load_dwordx2 v[64:65], %[l8], s[78:79] offset:0\n"\
      "global_load_dwordx2 v[66:67], %[l8], s[78:79] offset:512\n"\
      "global_load_dwordx2 v[68:69], %[l8], s[78:79] offset:1024\n"\
      "global_load_dwordx2 v[70:71], %[l8], s[78:79] offset:1536\n"\
      "global_load_dwordx2 v[72:73], %[l8], s[78:79] offset:2048\n"\
      "global_load_dwordx2 v[74:75], %[l8], s[78:79] offset:2560\n"\
      "global_load_dwordx2 v[76:77], %[l8], s[78:79] offset:3072\n"\
      "global_load_dwordx2 v[78:79], %[l8], s[78:79] offset:3584\n"\
      "global_load_dwordx2 v[80:81], %[l8], s[80:81] offset:0\n"\
      "global_load_dwordx2 v[82:83], %[l8], s[80:81] offset:512\n"\
      "global_load_dwordx2 v[84:85], %[l8], s[80:81] offset:1024\n"\
      "global_load_dwordx2 v[86:87], %[l8], s[80:81] offset:1536\n"\
      "global_load_dwordx2 v[88:89], %[l8], s[80:81] offset:2048\n"\
      "global_load_dwordx2 v[90:91], %[l8], s[80:81] offset:2560\n"\
      "global_load_dwordx2 v[92:93], %[l8], s[80:81] offset:3072\n"\
      "global_load_dwordx2 v[94:95], %[l8], s[80:81] offset:3584\n"\
      "global_load_dwordx2 v[96:97], %[l8], s[82:83] offset:0\n"\
      "global_load_dwordx2 v[98:99], %[l8], s[82:83] offset:512\n"\
      "global_load_dwordx2 v[100:101], %[l8], s[82:83] offset:1024\n"\
      "global_load_dwordx2 v[102:103], %[l8], s[82:83] offset:1536\n"\
      "global_load_dwordx2 v[104:105], %[l8], s[82:83] offset:2048\n"\
      "global_load_dwordx2 v[106:107], %[l8], s[82:83] offset:2560\n"\
      "global_load_dwordx2 v[108:109], %[l8], s[82:83] offset:3072\n"\
      "global_load_dwordx2 v[110:111], %[l8], s[82:83] offset:3584\n"\
      "global_load_dwordx2 v[112:113], %[l8], s[84:85] offset:0\n"\
      "global_load_dwordx2 v[114:115], %[l8], s[84:85] offset:512\n"\
      "global_load_dwordx2 v[116:117], %[l8], s[84:85] offset:1024\n"\
      "global_load_dwordx2 v[118:119], %[l8], s[84:85] offset:1536\n"\
      "global_load_dwordx2 v[120:121], %[l8], s[84:85] offset:2048\n"\
      "global_load_dwordx2 v[122:123], %[l8], s[84:85] offset:2560\n"\
      "global_load_dwordx2 v[124:125], %[l8], s[84:85] offset:3072\n"\
      "global_load_dwordx2 v[126:127], %[l8], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_lshlrev_b64 v[8:9], 16, v[96:97]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[98:99]\n"\
      "v_lshrrev_b32 v12, 16, v97\n"\
      "v_lshrrev_b32 v20, 16, v99\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mov_b32 v14, 0\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v96, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v97, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v67, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v96, s[36:37], v96, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[100:101]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[102:103]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[104:105]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[106:107]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[108:109]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[110:111]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[112:113]\n"\
      "v_lshrrev_b32 v28, 16, v101\n"\
      "v_lshrrev_b32 v36, 16, v103\n"\
      "v_lshrrev_b32 v44, 16, v105\n"\
      "v_lshrrev_b32 v52, 16, v107\n"\
      "v_lshrrev_b32 v60, 16, v109\n"\
      "v_lshrrev_b32 v12, 16, v111\n"\
      "v_lshrrev_b32 v20, 16, v113\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v80, v18\n"\
      "v_sub_co_u32_e64 v100, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v102, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v104, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v106, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v108, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v110, s[36:37], v78, v10\n"\
      "v_sub_co_u32_e64 v112, s[42:43], v80, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v81, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v101, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v103, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v105, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v107, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v109, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v111, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v113, s[44:45], v81, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v100, s[48:49], v100, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v102, s[54:55], v102, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v104, s[60:61], v104, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v106, s[66:67], v106, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v108, s[72:73], v108, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v110, s[36:37], v110, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v112, s[42:43], v112, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[114:115]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[116:117]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[118:119]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[120:121]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[122:123]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[124:125]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[126:127]\n"\
      "v_lshrrev_b32 v28, 16, v115\n"\
      "v_lshrrev_b32 v36, 16, v117\n"\
      "v_lshrrev_b32 v44, 16, v119\n"\
      "v_lshrrev_b32 v52, 16, v121\n"\
      "v_lshrrev_b32 v60, 16, v123\n"\
      "v_lshrrev_b32 v12, 16, v125\n"\
      "v_lshrrev_b32 v20, 16, v127\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v82, v26\n"\
      "v_sub_co_u32_e64 v114, s[48:49], v82, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v84, v34\n"\
      "v_sub_co_u32_e64 v116, s[54:55], v84, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v86, v42\n"\
      "v_sub_co_u32_e64 v118, s[60:61], v86, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v88, v50\n"\
      "v_sub_co_u32_e64 v120, s[66:67], v88, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v90, v58\n"\
      "v_sub_co_u32_e64 v122, s[72:73], v90, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_sub_co_u32_e64 v124, s[36:37], v92, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v94, v18\n"\
      "v_sub_co_u32_e64 v126, s[42:43], v94, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v83, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v115, s[50:51], v83, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v85, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v117, s[56:57], v85, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v87, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v119, s[62:63], v87, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v89, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v121, s[68:69], v89, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v91, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v123, s[74:75], v91, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v125, s[38:39], v93, v11, s[36:37]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v95, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v127, s[44:45], v95, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v114, s[48:49], v114, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v116, s[54:55], v116, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v118, s[60:61], v118, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v120, s[66:67], v120, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v122, s[72:73], v122, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v124, s[36:37], v124, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v126, s[42:43], v126, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v127, s[24:25], v127, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[80:81]\n"\
      "v_lshlrev_b64 v[16:17], 24, v[82:83]\n"\
      "v_lshrrev_b32 v12, 8, v81\n"\
      "v_lshrrev_b32 v20, 8, v83\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v82, s[42:43], v66, v18\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v80, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[44:45], v67, v19, s[42:43]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v82, s[42:43], v82, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v80, s[36:37], v80, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v12, s[36:37]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[112:113]\n"\
      "v_lshlrev_b32 v20, 8, v112\n"\
      "v_lshlrev_b64 v[24:25], 24, v[84:85]\n"\
      "v_lshlrev_b64 v[32:33], 24, v[86:87]\n"\
      "v_lshlrev_b64 v[40:41], 24, v[88:89]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[94:95]\n"\
      "v_lshrrev_b32 v28, 8, v85\n"\
      "v_lshrrev_b32 v36, 8, v87\n"\
      "v_lshrrev_b32 v44, 8, v89\n"\
      "v_lshrrev_b32 v52, 8, v91\n"\
      "v_lshrrev_b32 v60, 8, v93\n"\
      "v_lshrrev_b32 v12, 8, v95\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_sub_co_u32_e64 v84, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v86, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v78, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v96, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v85, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v87, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v97, s[44:45], v97, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v84, s[48:49], v84, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v86, s[54:55], v86, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v96, s[42:43], v96, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v20, s[42:43]\n"\
      "v_lshrrev_b64 v[24:25], 24, v[114:115]\n"\
      "v_lshrrev_b64 v[32:33], 24, v[116:117]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[118:119]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 24, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 24, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[126:127]\n"\
      "v_lshlrev_b32 v28, 8, v114\n"\
      "v_lshlrev_b32 v36, 8, v116\n"\
      "v_lshlrev_b32 v44, 8, v118\n"\
      "v_lshlrev_b32 v52, 8, v120\n"\
      "v_lshlrev_b32 v60, 8, v122\n"\
      "v_lshlrev_b32 v12, 8, v124\n"\
      "v_lshlrev_b32 v20, 8, v126\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v28, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_sub_co_u32_e64 v27, s[48:49], v27, v28\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[48:49]\n"\
      "v_addc_co_u32_e64 v26, s[50:51], v26, 0, s[48:49]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v29, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v104, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v106, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v108, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v110, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_sub_co_u32_e64 v98, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v100, s[54:55], v100, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v102, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v105, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v104, s[66:67], v104, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v107, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v106, s[72:73], v106, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v109, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v108, s[36:37], v108, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v111, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v110, s[42:43], v110, v18\n"\
      "v_subb_co_u32_e64 v99, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v101, s[56:57], v101, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v103, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v105, s[68:69], v105, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v107, s[74:75], v107, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v109, s[38:39], v109, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v111, s[44:45], v111, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v98, s[48:49], v98, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v100, s[54:55], v100, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v102, s[60:61], v102, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v104, s[66:67], v104, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v106, s[72:73], v106, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v108, s[36:37], v108, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v110, s[42:43], v110, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[116:117], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 12, v[72:73]\n"\
      "v_lshlrev_b64 v[16:17], 12, v[74:75]\n"\
      "v_lshrrev_b32 v12, 20, v73\n"\
      "v_lshrrev_b32 v20, 20, v75\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v72, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v74, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v73, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v75, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 28, v[88:89]\n"\
      "v_lshrrev_b32 v44, 4, v89\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v72, s[36:37], v72, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v74, s[42:43], v74, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshlrev_b64 v[48:49], 28, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 28, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 28, v[94:95]\n"\
      "v_lshlrev_b64 v[16:17], 4, v[104:105]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshrrev_b32 v52, 4, v91\n"\
      "v_lshrrev_b32 v60, 4, v93\n"\
      "v_lshrrev_b32 v12, 4, v95\n"\
      "v_lshrrev_b32 v20, 28, v105\n"\
      "v_lshlrev_b64 v[24:25], 12, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 12, v[78:79]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 20, v77\n"\
      "v_lshrrev_b32 v36, 20, v79\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v81, v43, s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v84, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v86, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v82, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v84, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v86, v10\n"\
      "v_sub_co_u32_e64 v104, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v85, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v87, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v85, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v87, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v105, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 4, v[106:107]\n"\
      "v_lshlrev_b64 v[32:33], 4, v[108:109]\n"\
      "v_lshlrev_b64 v[40:41], 4, v[110:111]\n"\
      "v_lshrrev_b32 v28, 28, v107\n"\
      "v_lshrrev_b32 v36, 28, v109\n"\
      "v_lshrrev_b32 v44, 28, v111\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v104, s[42:43], v104, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 12, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 12, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 12, v[126:127]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 20, v120\n"\
      "v_lshlrev_b32 v60, 20, v122\n"\
      "v_lshlrev_b32 v12, 20, v124\n"\
      "v_lshlrev_b32 v20, 20, v126\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v116, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v118, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v106, s[48:49], v98, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_sub_co_u32_e64 v108, s[54:55], v100, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_sub_co_u32_e64 v110, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v112, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v114, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v117, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v116, s[36:37], v116, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v119, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v118, s[42:43], v118, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v107, s[50:51], v99, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v109, s[56:57], v101, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v111, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v113, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v115, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v117, s[38:39], v117, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v119, s[44:45], v119, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v106, s[48:49], v106, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v108, s[54:55], v108, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v110, s[60:61], v110, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v112, s[66:67], v112, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v114, s[72:73], v114, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v116, s[36:37], v116, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v118, s[42:43], v118, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 6, v[68:69]\n"\
      "v_lshrrev_b32 v12, 26, v69\n"\
      "v_lshlrev_b64 v[16:17], 6, v[70:71]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 26, v71\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_lshlrev_b64 v[24:25], 22, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 22, v[78:79]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshrrev_b32 v28, 10, v77\n"\
      "v_lshrrev_b32 v36, 10, v79\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v68, s[36:37], v64, v10\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v66, v18\n"\
      "v_subb_co_u32_e64 v69, s[38:39], v65, v11, s[36:37]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshrrev_b64 v[56:57], 18, v[92:93]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_lshlrev_b32 v60, 14, v92\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 30, v[84:85]\n"\
      "v_lshlrev_b64 v[48:49], 30, v[86:87]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v68, s[36:37], v68, 0, s[38:39]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v44, 2, v85\n"\
      "v_lshrrev_b32 v52, 2, v87\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_lshrrev_b64 v[8:9], 18, v[94:95]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_lshlrev_b32 v12, 14, v94\n"\
      "v_lshlrev_b64 v[16:17], 18, v[100:101]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 14, v101\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v82, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v88, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v89, s[74:75], v89, v59, s[72:73]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v90, v10\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v88, s[72:73], v88, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v74, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v74, v34\n"\
      "v_sub_co_u32_e64 v84, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v91, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v90, v10\n"\
      "v_sub_co_u32_e64 v100, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v60, s[72:73]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v75, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v72, v26\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v75, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v85, s[62:63], v81, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v91, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v101, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 10, v[116:117]\n"\
      "v_lshlrev_b64 v[56:57], 10, v[118:119]\n"\
      "v_lshrrev_b32 v52, 22, v117\n"\
      "v_lshrrev_b32 v60, 22, v119\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v73, v27, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v84, s[60:61], v84, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v100, s[42:43], v100, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_lshrrev_b64 v[32:33], 30, v[108:109]\n"\
      "v_lshrrev_b64 v[40:41], 30, v[110:111]\n"\
      "v_lshrrev_b64 v[8:9], 6, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 6, v[126:127]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_lshlrev_b32 v36, 2, v108\n"\
      "v_lshlrev_b32 v44, 2, v110\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v12, 26, v124\n"\
      "v_lshlrev_b32 v20, 26, v126\n"\
      "v_lshlrev_b64 v[24:25], 18, v[102:103]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 14, v103\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v106, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v122, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v104, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v107, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v106, s[60:61], v106, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v116, s[66:67], v112, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_sub_co_u32_e64 v118, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v120, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v123, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v122, s[42:43], v122, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v105, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v107, s[62:63], v107, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v117, s[68:69], v113, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v119, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v121, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v123, s[44:45], v123, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v104, s[54:55], v104, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v106, s[60:61], v106, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v116, s[66:67], v116, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v118, s[72:73], v118, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v120, s[36:37], v120, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v122, s[42:43], v122, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[16:17], 19, v[70:71]\n"\
      "v_lshlrev_b64 v[8:9], 3, v[66:67]\n"\
      "v_lshrrev_b32 v20, 13, v71\n"\
      "v_lshrrev_b32 v12, 29, v67\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_sub_co_u32_e64 v66, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_subb_co_u32_e64 v67, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v66, s[36:37], v66, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v68, v18\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v68, v18\n"\
      "v_lshlrev_b64 v[48:49], 31, v[86:87]\n"\
      "v_lshlrev_b64 v[56:57], 7, v[90:91]\n"\
      "v_lshrrev_b64 v[32:33], 21, v[78:79]\n"\
      "v_lshrrev_b32 v52, 1, v87\n"\
      "v_lshrrev_b32 v60, 25, v91\n"\
      "v_lshrrev_b64 v[8:9], 9, v[94:95]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v69, v19, s[46:47]\n"\
      "v_lshlrev_b32 v36, 11, v78\n"\
      "v_lshlrev_b32 v12, 23, v94\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v69, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 27, v[74:75]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_lshrrev_b32 v28, 5, v75\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 15, v[82:83]\n"\
      "v_lshlrev_b64 v[16:17], 9, v[98:99]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_lshrrev_b32 v44, 17, v83\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v20, 23, v99\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v76, v34\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v77, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v76, v34\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v92, v10\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v73, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v77, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v93, v11, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v37, 1, v[32:33]\n"\
      "v_sub_co_u32_e64 v82, s[60:61], v80, v42\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v84, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[62:63], v81, v43, s[60:61]\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v84, v50\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v89, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 25, v[102:103]\n"\
      "v_lshlrev_b64 v[32:33], 1, v[106:107]\n"\
      "v_lshlrev_b64 v[8:9], 13, v[122:123]\n"\
      "v_lshrrev_b32 v28, 7, v103\n"\
      "v_lshrrev_b32 v36, 31, v107\n"\
      "v_lshrrev_b32 v12, 19, v123\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v85, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v82, s[60:61], v82, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v85, v51, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v44, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshrrev_b64 v[40:41], 15, v[110:111]\n"\
      "v_lshrrev_b64 v[56:57], 27, v[118:119]\n"\
      "v_lshrrev_b64 v[16:17], 3, v[126:127]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshlrev_b32 v44, 17, v110\n"\
      "v_lshlrev_b32 v60, 5, v118\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_lshlrev_b32 v20, 29, v126\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshlrev_b64 v[48:49], 21, v[114:115]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v52, 11, v115\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v108, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v116, v58\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v124, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v100, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v100, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_sub_co_u32_e64 v106, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v109, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v108, s[60:61], v108, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v114, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v117, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v116, s[72:73], v116, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_sub_co_u32_e64 v122, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v125, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v124, s[42:43], v124, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v101, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v101, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v107, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v109, s[62:63], v109, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v115, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v117, s[74:75], v117, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v123, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v125, s[44:45], v125, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v106, s[54:55], v106, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v108, s[60:61], v108, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v114, s[66:67], v114, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v116, s[72:73], v116, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v122, s[36:37], v122, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v124, s[42:43], v124, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[86:87] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[86:87] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[86:87] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[86:87] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[86:87] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[86:87] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[86:87] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[86:87] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v64, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v66, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v64, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v66, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v65, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v65, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v67, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v67, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v68, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v64, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v65, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v66, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v67, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v70, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v72, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v68, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v70, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v72, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v69, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v69, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v71, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v71, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v73, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v73, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v68, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v69, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v70, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v71, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v72, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v73, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v74, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v76, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v78, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v74, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v76, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v78, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v75, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v75, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v77, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v77, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v79, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v79, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v74, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v75, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v76, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v77, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v78, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v79, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[88:89] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[88:89] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[88:89] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[88:89] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[88:89] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[88:89] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[88:89] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[88:89] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v80, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v82, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v80, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v82, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v81, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v81, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v83, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v83, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v84, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v80, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v81, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v82, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v83, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v86, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v88, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v84, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v86, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v88, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v85, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v85, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v87, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v87, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v89, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v89, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v84, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v85, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v86, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v87, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v88, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v89, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v90, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v92, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v94, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v90, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v92, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v94, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v91, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v91, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v93, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v93, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v95, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v95, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v90, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v91, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v92, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v93, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v94, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v95, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[90:91] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[90:91] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[90:91] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[90:91] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[90:91] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[90:91] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[90:91] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[90:91] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v96, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v98, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v96, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v98, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v97, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v97, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v99, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v99, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v100, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v96, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v97, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v98, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v99, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v102, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v104, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v100, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v102, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v104, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v101, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v101, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v103, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v103, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v105, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v105, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v100, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v101, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v102, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v103, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v104, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v106, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v108, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v110, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v106, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v108, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v110, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v107, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v107, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v109, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v109, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v111, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v111, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v106, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v107, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v108, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v109, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v110, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v111, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[92:93] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[92:93] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[92:93] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[92:93] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[92:93] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[92:93] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[92:93] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[92:93] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v112, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v114, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v112, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v114, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v113, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v113, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v115, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v115, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v116, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v112, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v113, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v114, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v115, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v118, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v120, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v116, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v118, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v120, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v117, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v117, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v119, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v119, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v121, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v121, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v116, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v117, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v118, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v119, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v120, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v121, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v122, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v124, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v126, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v122, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v124, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v126, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v123, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v123, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v125, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v125, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v127, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v127, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v122, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v123, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v124, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v125, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v126, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v127, v37, v41, s[44:45]\n"\
      "s_mov_b32 exec_lo, -1\n"\
      "s_mov_b32 exec_hi, 0\n"\
      "ds_write_b64 %[t1w], v[64:65] offset:0\n"\
      "ds_write_b64 %[t1w], v[66:67] offset:272\n"\
      "ds_write_b64 %[t1w], v[68:69] offset:544\n"\
      "ds_write_b64 %[t1w], v[70:71] offset:816\n"\
      "ds_write_b64 %[t1w], v[72:73] offset:1088\n"\
      "ds_write_b64 %[t1w], v[74:75] offset:1360\n"\
      "ds_write_b64 %[t1w], v[76:77] offset:1632\n"\
      "ds_write_b64 %[t1w], v[78:79] offset:1904\n"\
      "ds_write_b64 %[t1w], v[80:81] offset:2176\n"\
      "ds_write_b64 %[t1w], v[82:83] offset:2448\n"\
      "ds_write_b64 %[t1w], v[84:85] offset:2720\n"\
      "ds_write_b64 %[t1w], v[86:87] offset:2992\n"\
      "ds_write_b64 %[t1w], v[88:89] offset:3264\n"\
      "ds_write_b64 %[t1w], v[90:91] offset:3536\n"\
      "ds_write_b64 %[t1w], v[92:93] offset:3808\n"\
      "ds_write_b64 %[t1w], v[94:95] offset:4080\n"\
      "ds_write_b64 %[t1w], v[96:97] offset:4352\n"\
      "ds_write_b64 %[t1w], v[98:99] offset:4624\n"\
      "ds_write_b64 %[t1w], v[100:101] offset:4896\n"\
      "ds_write_b64 %[t1w], v[102:103] offset:5168\n"\
      "ds_write_b64 %[t1w], v[104:105] offset:5440\n"\
      "ds_write_b64 %[t1w], v[106:107] offset:5712\n"\
      "ds_write_b64 %[t1w], v[108:109] offset:5984\n"\
      "ds_write_b64 %[t1w], v[110:111] offset:6256\n"\
      "ds_write_b64 %[t1w], v[112:113] offset:6528\n"\
      "ds_write_b64 %[t1w], v[114:115] offset:6800\n"\
      "ds_write_b64 %[t1w], v[116:117] offset:7072\n"\
      "ds_write_b64 %[t1w], v[118:119] offset:7344\n"\
      "ds_write_b64 %[t1w], v[120:121] offset:7616\n"\
      "ds_write_b64 %[t1w], v[122:123] offset:7888\n"\
      "ds_write_b64 %[t1w], v[124:125] offset:8160\n"\
      "ds_write_b64 %[t1w], v[126:127] offset:8432\n"\
      "s_mov_b64 exec, s[22:23]\n"\
      "ds_read_b64 v[8:9], %[t1r] offset:0\n"\
      "ds_read_b64 v[10:11], %[t1r] offset:16\n"\
      "ds_read_b64 v[12:13], %[t1r] offset:32\n"\
      "ds_read_b64 v[14:15], %[t1r] offset:48\n"\
      "ds_read_b64 v[16:17], %[t1r] offset:64\n"\
      "ds_read_b64 v[18:19], %[t1r] offset:80\n"\
      "ds_read_b64 v[20:21], %[t1r] offset:96\n"\
      "ds_read_b64 v[22:23], %[t1r] offset:112\n"\
      "ds_read_b64 v[24:25], %[t1r] offset:128\n"\
      "ds_read_b64 v[26:27], %[t1r] offset:144\n"\
      "ds_read_b64 v[28:29], %[t1r] offset:160\n"\
      "ds_read_b64 v[30:31], %[t1r] offset:176\n"\
      "ds_read_b64 v[32:33], %[t1r] offset:192\n"\
      "ds_read_b64 v[34:35], %[t1r] offset:208\n"\
      "ds_read_b64 v[36:37], %[t1r] offset:224\n"\
      "ds_read_b64 v[38:39], %[t1r] offset:240\n"\
      "s_mov_b32 exec_lo, 0\n"\
      "s_mov_b32 exec_hi, -1\n"\
      "ds_write_b64 %[t1w], v[64:65] offset:0\n"\
      "ds_write_b64 %[t1w], v[66:67] offset:272\n"\
      "ds_write_b64 %[t1w], v[68:69] offset:544\n"\
      "ds_write_b64 %[t1w], v[70:71] offset:816\n"\
      "ds_write_b64 %[t1w], v[72:73] offset:1088\n"\
      "ds_write_b64 %[t1w], v[74:75] offset:1360\n"\
      "ds_write_b64 %[t1w], v[76:77] offset:1632\n"\
      "ds_write_b64 %[t1w], v[78:79] offset:1904\n"\
      "ds_write_b64 %[t1w], v[80:81] offset:2176\n"\
      "ds_write_b64 %[t1w], v[82:83] offset:2448\n"\
      "ds_write_b64 %[t1w], v[84:85] offset:2720\n"\
      "ds_write_b64 %[t1w], v[86:87] offset:2992\n"\
      "ds_write_b64 %[t1w], v[88:89] offset:3264\n"\
      "ds_write_b64 %[t1w], v[90:91] offset:3536\n"\
      "ds_write_b64 %[t1w], v[92:93] offset:3808\n"\
      "ds_write_b64 %[t1w], v[94:95] offset:4080\n"\
      "ds_write_b64 %[t1w], v[96:97] offset:4352\n"\
      "ds_write_b64 %[t1w], v[98:99] offset:4624\n"\
      "ds_write_b64 %[t1w], v[100:101] offset:4896\n"\
      "ds_write_b64 %[t1w], v[102:103] offset:5168\n"\
      "ds_write_b64 %[t1w], v[104:105] offset:5440\n"\
      "ds_write_b64 %[t1w], v[106:107] offset:5712\n"\
      "ds_write_b64 %[t1w], v[108:109] offset:5984\n"\
      "ds_write_b64 %[t1w], v[110:111] offset:6256\n"\
      "ds_write_b64 %[t1w], v[112:113] offset:6528\n"\
      "ds_write_b64 %[t1w], v[114:115] offset:6800\n"\
      "ds_write_b64 %[t1w], v[116:117] offset:7072\n"\
      "ds_write_b64 %[t1w], v[118:119] offset:7344\n"\
      "ds_write_b64 %[t1w], v[120:121] offset:7616\n"\
      "ds_write_b64 %[t1w], v[122:123] offset:7888\n"\
      "ds_write_b64 %[t1w], v[124:125] offset:8160\n"\
      "ds_write_b64 %[t1w], v[126:127] offset:8432\n"\
      "s_mov_b64 exec, s[22:23]\n"\
      "s_waitcnt lgkmcnt(0)\n"\
      "ds_read_b64 v[64:65], %[t1r] offset:0\n"\
      "ds_read_b64 v[66:67], %[t1r] offset:16\n"\
      "ds_read_b64 v[68:69], %[t1r] offset:32\n"\
      "ds_read_b64 v[70:71], %[t1r] offset:48\n"\
      "ds_read_b64 v[72:73], %[t1r] offset:64\n"\
      "ds_read_b64 v[74:75], %[t1r] offset:80\n"\
      "ds_read_b64 v[76:77], %[t1r] offset:96\n"\
      "ds_read_b64 v[78:79], %[t1r] offset:112\n"\
      "ds_read_b64 v[80:81], %[t1r] offset:128\n"\
      "ds_read_b64 v[82:83], %[t1r] offset:144\n"\
      "ds_read_b64 v[84:85], %[t1r] offset:160\n"\
      "ds_read_b64 v[86:87], %[t1r] offset:176\n"\
      "ds_read_b64 v[88:89], %[t1r] offset:192\n"\
      "ds_read_b64 v[90:91], %[t1r] offset:208\n"\
      "ds_read_b64 v[92:93], %[t1r] offset:224\n"\
      "ds_read_b64 v[94:95], %[t1r] offset:240\n"\
      "s_waitcnt lgkmcnt(0)\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[64:65]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[66:67]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[68:69]\n"\
      "v_cndmask_b32_e64 v42, v64, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v50, v66, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v43, v65, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_cndmask_b32_e64 v51, v67, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v64, s[36:37], v8, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v66, s[42:43], v10, v50\n"\
      "v_subb_co_u32_e64 v65, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v67, s[44:45], v11, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v64, s[36:37], v64, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v66, s[42:43], v66, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[70:71]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[72:73]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[74:75]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[76:77]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[78:79]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[80:81]\n"\
      "v_cndmask_b32_e64 v58, v68, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v70, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v72, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v114, v74, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v122, v76, v120, s[74:75]\n"\
      "v_cndmask_b32_e64 v42, v78, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v50, v80, v48, s[44:45]\n"\
      "v_addc_co_u32_e64 v65, s[24:25], v65, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v59, v69, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v12, v58\n"\
      "v_cndmask_b32_e64 v99, v71, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v14, v98\n"\
      "v_cndmask_b32_e64 v107, v73, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v16, v106\n"\
      "v_cndmask_b32_e64 v115, v75, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v18, v114\n"\
      "v_cndmask_b32_e64 v123, v77, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v20, v122\n"\
      "v_cndmask_b32_e64 v43, v79, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v22, v42\n"\
      "v_cndmask_b32_e64 v51, v81, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v24, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v13, v59, s[52:53]\n"\
      "v_sub_co_u32_e64 v68, s[48:49], v12, v58\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v15, v99, s[58:59]\n"\
      "v_sub_co_u32_e64 v70, s[54:55], v14, v98\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v17, v107, s[64:65]\n"\
      "v_sub_co_u32_e64 v72, s[60:61], v16, v106\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v19, v115, s[70:71]\n"\
      "v_sub_co_u32_e64 v74, s[66:67], v18, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v21, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v76, s[72:73], v20, v122\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v23, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v78, s[36:37], v22, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v25, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v80, s[42:43], v24, v50\n"\
      "v_subb_co_u32_e64 v69, s[50:51], v13, v59, s[48:49]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_subb_co_u32_e64 v71, s[56:57], v15, v99, s[54:55]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_subb_co_u32_e64 v73, s[62:63], v17, v107, s[60:61]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_subb_co_u32_e64 v75, s[68:69], v19, v115, s[66:67]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_subb_co_u32_e64 v77, s[74:75], v21, v123, s[72:73]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_subb_co_u32_e64 v79, s[38:39], v23, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[44:45], v25, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v68, s[48:49], v68, 0, s[50:51]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v61, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v70, s[54:55], v70, 0, s[56:57]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v72, s[60:61], v72, 0, s[62:63]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v109, 1, v[104:105]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v74, s[66:67], v74, 0, s[68:69]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v117, 1, v[112:113]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v76, s[72:73], v76, 0, s[74:75]\n"\
      "v_mad_u64_u32 v[20:21], s[24:25], v125, 1, v[120:121]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v78, s[36:37], v78, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v80, s[42:43], v80, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[82:83]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[84:85]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[86:87]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[88:89]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[90:91]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[92:93]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[94:95]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v108, s[60:61]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, v82, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v84, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v86, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v114, v88, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v122, v90, v120, s[74:75]\n"\
      "v_cndmask_b32_e64 v42, v92, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v50, v94, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v59, v83, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v26, v58\n"\
      "v_sub_co_u32_e64 v82, s[48:49], v26, v58\n"\
      "v_cndmask_b32_e64 v99, v85, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v28, v98\n"\
      "v_sub_co_u32_e64 v84, s[54:55], v28, v98\n"\
      "v_cndmask_b32_e64 v107, v87, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v30, v106\n"\
      "v_sub_co_u32_e64 v86, s[60:61], v30, v106\n"\
      "v_cndmask_b32_e64 v115, v89, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v32, v114\n"\
      "v_sub_co_u32_e64 v88, s[66:67], v32, v114\n"\
      "v_cndmask_b32_e64 v123, v91, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v34, v122\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v34, v122\n"\
      "v_cndmask_b32_e64 v43, v93, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v36, v42\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v36, v42\n"\
      "v_cndmask_b32_e64 v51, v95, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v38, v50\n"\
      "v_sub_co_u32_e64 v94, s[42:43], v38, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v27, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v83, s[50:51], v27, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v29, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v85, s[56:57], v29, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v31, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v87, s[62:63], v31, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v33, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v89, s[68:69], v33, v115, s[66:67]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v35, v123, s[76:77]\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v35, v123, s[72:73]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v37, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v37, v43, s[36:37]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v39, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v95, s[44:45], v39, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v82, s[48:49], v82, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v84, s[54:55], v84, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v86, s[60:61], v86, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v88, s[66:67], v88, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v94, s[42:43], v94, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[24:25]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_cndmask_b32_e64 v50, v26, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v51, v27, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_sub_co_u32_e64 v26, s[42:43], v10, v50\n"\
      "v_cndmask_b32_e64 v42, v24, v40, s[38:39]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v27, s[44:45], v11, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v43, v25, v41, s[38:39]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v26, s[42:43], v26, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[80:81]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v52, s[42:43]\n"\
      "v_lshrrev_b32 v52, 16, v81\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_sub_co_u32_e64 v24, s[36:37], v8, v42\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_subb_co_u32_e64 v25, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_mov_b32 v55, v48\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v24, s[36:37], v24, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[28:29]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[36:37]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[38:39]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v58, v28, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v30, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v32, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v114, v34, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v122, v36, v120, s[74:75]\n"\
      "v_cndmask_b32_e64 v42, v38, v40, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_addc_co_u32_e64 v25, s[24:25], v25, v44, s[36:37]\n"\
      "v_cndmask_b32_e64 v59, v29, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v12, v58\n"\
      "v_cndmask_b32_e64 v99, v31, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v14, v98\n"\
      "v_cndmask_b32_e64 v107, v33, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v16, v106\n"\
      "v_cndmask_b32_e64 v115, v35, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v18, v114\n"\
      "v_cndmask_b32_e64 v123, v37, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v20, v122\n"\
      "v_cndmask_b32_e64 v43, v39, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v22, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_sub_co_u32_e64 v28, s[48:49], v12, v58\n"\
      "v_sub_co_u32_e64 v30, s[54:55], v14, v98\n"\
      "v_sub_co_u32_e64 v32, s[60:61], v16, v106\n"\
      "v_sub_co_u32_e64 v34, s[66:67], v18, v114\n"\
      "v_sub_co_u32_e64 v36, s[72:73], v20, v122\n"\
      "v_sub_co_u32_e64 v38, s[36:37], v22, v42\n"\
      "v_sub_co_u32_e64 v80, s[42:43], v64, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v13, v59, s[52:53]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v15, v99, s[58:59]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v17, v107, s[64:65]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v19, v115, s[70:71]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v21, v123, s[76:77]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v23, v43, s[40:41]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v29, s[50:51], v13, v59, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[56:57], v15, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v33, s[62:63], v17, v107, s[60:61]\n"\
      "v_subb_co_u32_e64 v35, s[68:69], v19, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v37, s[74:75], v21, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v39, s[38:39], v23, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v81, s[44:45], v65, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v28, s[48:49], v28, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v30, s[54:55], v30, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v32, s[60:61], v32, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v34, s[66:67], v34, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v36, s[72:73], v36, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v38, s[36:37], v38, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v80, s[42:43], v80, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v109, 1, v[104:105]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v117, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[20:21], s[24:25], v125, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v29, s[24:25], v29, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v31, s[24:25], v31, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v33, s[24:25], v33, v108, s[60:61]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v37, s[24:25], v37, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v39, s[24:25], v39, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v52, s[42:43]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[82:83]\n"\
      "v_lshlrev_b64 v[96:97], 16, v[84:85]\n"\
      "v_lshlrev_b64 v[104:105], 16, v[86:87]\n"\
      "v_lshlrev_b64 v[112:113], 16, v[88:89]\n"\
      "v_lshlrev_b64 v[120:121], 16, v[90:91]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[92:93]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[94:95]\n"\
      "v_lshrrev_b32 v60, 16, v83\n"\
      "v_lshrrev_b32 v100, 16, v85\n"\
      "v_lshrrev_b32 v108, 16, v87\n"\
      "v_lshrrev_b32 v116, 16, v89\n"\
      "v_lshrrev_b32 v124, 16, v91\n"\
      "v_lshrrev_b32 v44, 16, v93\n"\
      "v_lshrrev_b32 v52, 16, v95\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v100, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v108, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v102, 0\n"\
      "v_mov_b32 v103, v96\n"\
      "v_mov_b32 v110, 0\n"\
      "v_mov_b32 v111, v104\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v97, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v105, -1, v[110:111]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v66, v58\n"\
      "v_sub_co_u32_e64 v82, s[48:49], v66, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v68, v98\n"\
      "v_sub_co_u32_e64 v84, s[54:55], v68, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v70, v106\n"\
      "v_sub_co_u32_e64 v86, s[60:61], v70, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v72, v114\n"\
      "v_sub_co_u32_e64 v88, s[66:67], v72, v114\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v74, v122\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v74, v122\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v76, v42\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v76, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v78, v50\n"\
      "v_sub_co_u32_e64 v94, s[42:43], v78, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v67, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v83, s[50:51], v67, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v69, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v85, s[56:57], v69, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v71, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v87, s[62:63], v71, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v73, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v89, s[68:69], v73, v115, s[66:67]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v75, v123, s[76:77]\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v75, v123, s[72:73]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v77, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v77, v43, s[36:37]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v79, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v95, s[44:45], v79, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v82, s[48:49], v82, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v84, s[54:55], v84, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v86, s[60:61], v86, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v88, s[66:67], v88, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v94, s[42:43], v94, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshlrev_b64 v[104:105], 16, v[32:33]\n"\
      "v_cndmask_b32_e64 v42, v16, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v17, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_sub_co_u32_e64 v16, s[36:37], v8, v42\n"\
      "v_cndmask_b32_e64 v50, v18, v48, s[44:45]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v17, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v51, v19, v49, s[44:45]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v16, s[36:37], v16, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_addc_co_u32_e64 v17, s[24:25], v17, v44, s[36:37]\n"\
      "v_sub_co_u32_e64 v18, s[42:43], v10, v50\n"\
      "v_lshlrev_b64 v[112:113], 16, v[34:35]\n"\
      "v_lshlrev_b64 v[120:121], 16, v[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[38:39]\n"\
      "v_lshrrev_b32 v108, 16, v33\n"\
      "v_lshrrev_b32 v116, 16, v35\n"\
      "v_lshrrev_b32 v124, 16, v37\n"\
      "v_lshrrev_b32 v44, 16, v39\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v19, s[44:45], v11, v51, s[42:43]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v44, -1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v18, s[42:43], v18, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v108, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[72:73]\n"\
      "v_mov_b32 v110, 0\n"\
      "v_mov_b32 v111, v104\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_lshrrev_b32 v52, 8, v73\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v105, -1, v[110:111]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[22:23]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v58, v20, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v22, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v26, v114\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v28, v122\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v30, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_sub_co_u32_e64 v34, s[66:67], v26, v114\n"\
      "v_sub_co_u32_e64 v36, s[72:73], v28, v122\n"\
      "v_sub_co_u32_e64 v38, s[36:37], v30, v42\n"\
      "v_sub_co_u32_e64 v72, s[42:43], v64, v50\n"\
      "v_cndmask_b32_e64 v59, v21, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v12, v58\n"\
      "v_cndmask_b32_e64 v99, v23, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v14, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v24, v106\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v27, v115, s[70:71]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v29, v123, s[76:77]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v31, v43, s[40:41]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v20, s[48:49], v12, v58\n"\
      "v_sub_co_u32_e64 v22, s[54:55], v14, v98\n"\
      "v_sub_co_u32_e64 v32, s[60:61], v24, v106\n"\
      "v_subb_co_u32_e64 v35, s[68:69], v27, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v37, s[74:75], v29, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v39, s[38:39], v31, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v73, s[44:45], v65, v51, s[42:43]\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v13, v59, s[52:53]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v15, v99, s[58:59]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v25, v107, s[64:65]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v21, s[50:51], v13, v59, s[48:49]\n"\
      "v_subb_co_u32_e64 v23, s[56:57], v15, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v33, s[62:63], v25, v107, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v34, s[66:67], v34, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v36, s[72:73], v36, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v38, s[36:37], v38, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v72, s[42:43], v72, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v117, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v125, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v20, s[48:49], v20, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v22, s[54:55], v22, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v32, s[60:61], v32, 0, s[62:63]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v37, s[24:25], v37, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v39, s[24:25], v39, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v109, 1, v[104:105]\n"\
      "v_lshrrev_b64 v[112:113], 24, v[88:89]\n"\
      "v_lshrrev_b64 v[120:121], 24, v[90:91]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[92:93]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[94:95]\n"\
      "v_addc_co_u32_e64 v21, s[24:25], v21, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v23, s[24:25], v23, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v33, s[24:25], v33, v108, s[60:61]\n"\
      "v_lshlrev_b32 v116, 8, v88\n"\
      "v_lshlrev_b32 v124, 8, v90\n"\
      "v_lshlrev_b32 v44, 8, v92\n"\
      "v_lshlrev_b32 v52, 8, v94\n"\
      "v_lshlrev_b64 v[56:57], 24, v[74:75]\n"\
      "v_lshlrev_b64 v[96:97], 24, v[76:77]\n"\
      "v_lshlrev_b64 v[104:105], 24, v[78:79]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v116, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v124, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_lshrrev_b32 v60, 8, v75\n"\
      "v_lshrrev_b32 v100, 8, v77\n"\
      "v_lshrrev_b32 v108, 8, v79\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_sub_co_u32_e64 v115, s[66:67], v115, v116\n"\
      "v_sub_co_u32_e64 v123, s[72:73], v123, v124\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[42:43], v51, v52\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v114, s[68:69], v114, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v122, s[74:75], v122, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v50, s[44:45], v50, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v117, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v80, v114\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v125, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v82, v122\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v84, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v86, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v66, v58\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v66, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v68, v98\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v68, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v70, v106\n"\
      "v_sub_co_u32_e64 v78, s[60:61], v70, v106\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v81, v115, s[70:71]\n"\
      "v_sub_co_u32_e64 v80, s[66:67], v80, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v83, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v82, s[72:73], v82, v122\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v85, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v84, s[36:37], v84, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v87, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v86, s[42:43], v86, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v67, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v67, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v69, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v69, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v71, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v79, s[62:63], v71, v107, s[60:61]\n"\
      "v_subb_co_u32_e64 v81, s[68:69], v81, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v83, s[74:75], v83, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v85, s[38:39], v85, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[44:45], v87, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v78, s[60:61], v78, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v80, s[66:67], v80, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v82, s[72:73], v82, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v84, s[36:37], v84, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v86, s[42:43], v86, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[12:13]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[20:21]\n"\
      "v_lshlrev_b64 v[96:97], 16, v[22:23]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[14:15]\n"\
      "v_lshrrev_b32 v60, 16, v21\n"\
      "v_lshrrev_b32 v100, 16, v23\n"\
      "v_cndmask_b32_e64 v42, v12, v40, s[38:39]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_cndmask_b32_e64 v50, v14, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v43, v13, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_sub_co_u32_e64 v12, s[36:37], v8, v42\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v51, v15, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v14, s[42:43], v10, v50\n"\
      "v_subb_co_u32_e64 v13, s[38:39], v9, v43, s[36:37]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v100, 1, v[98:99]\n"\
      "v_lshrrev_b64 v[120:121], 24, v[36:37]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_lshlrev_b32 v124, 8, v36\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v15, s[44:45], v11, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[104:105], 24, v[28:29]\n"\
      "v_lshlrev_b64 v[112:113], 24, v[30:31]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v12, s[36:37], v12, 0, s[38:39]\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v102, 0\n"\
      "v_mov_b32 v103, v96\n"\
      "v_lshrrev_b32 v108, 8, v29\n"\
      "v_lshrrev_b32 v116, 8, v31\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v124, 1, v[120:121]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v14, s[42:43], v14, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v97, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_addc_co_u32_e64 v13, s[24:25], v13, v44, s[36:37]\n"\
      "v_sub_co_u32_e64 v123, s[72:73], v123, v124\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v15, s[24:25], v15, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[38:39]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v122, s[74:75], v122, 0, s[72:73]\n"\
      "v_lshlrev_b32 v44, 8, v38\n"\
      "v_lshlrev_b64 v[48:49], 12, v[68:69]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshrrev_b32 v52, 20, v69\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v125, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v32, v122\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v18, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v24, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v26, v114\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_sub_co_u32_e64 v22, s[54:55], v18, v98\n"\
      "v_sub_co_u32_e64 v28, s[60:61], v24, v106\n"\
      "v_sub_co_u32_e64 v30, s[66:67], v26, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v33, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v32, s[72:73], v32, v122\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v19, v99, s[58:59]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v25, v107, s[64:65]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v27, v115, s[70:71]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v23, s[56:57], v19, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v29, s[62:63], v25, v107, s[60:61]\n"\
      "v_subb_co_u32_e64 v31, s[68:69], v27, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v33, s[74:75], v33, v123, s[72:73]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v34, v42\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v22, s[54:55], v22, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v28, s[60:61], v28, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v30, s[66:67], v30, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v32, s[72:73], v32, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v109, 1, v[104:105]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v117, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v35, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v34, s[36:37], v34, v42\n"\
      "v_sub_co_u32_e64 v68, s[42:43], v64, v50\n"\
      "v_addc_co_u32_e64 v23, s[24:25], v23, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v29, s[24:25], v29, v108, s[60:61]\n"\
      "v_addc_co_u32_e64 v31, s[24:25], v31, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v33, s[24:25], v33, v124, s[72:73]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v16, v58\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v20, s[48:49], v16, v58\n"\
      "v_subb_co_u32_e64 v35, s[38:39], v35, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v69, s[44:45], v65, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[96:97], 28, v[76:77]\n"\
      "v_lshlrev_b64 v[104:105], 28, v[78:79]\n"\
      "v_lshlrev_b64 v[112:113], 4, v[84:85]\n"\
      "v_lshlrev_b64 v[120:121], 4, v[86:87]\n"\
      "v_lshrrev_b32 v100, 4, v77\n"\
      "v_lshrrev_b32 v108, 4, v79\n"\
      "v_lshrrev_b32 v116, 28, v85\n"\
      "v_lshrrev_b32 v124, 28, v87\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v17, v59, s[52:53]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v21, s[50:51], v17, v59, s[48:49]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v34, s[36:37], v34, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v68, s[42:43], v68, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v20, s[48:49], v20, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v61, 1, v[56:57]\n"\
      "v_lshrrev_b64 v[40:41], 12, v[92:93]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[94:95]\n"\
      "v_addc_co_u32_e64 v21, s[24:25], v21, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v100, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v108, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_lshlrev_b32 v44, 20, v92\n"\
      "v_lshlrev_b32 v52, 20, v94\n"\
      "v_lshlrev_b64 v[56:57], 12, v[70:71]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_lshrrev_b32 v60, 20, v71\n"\
      "v_mov_b32 v102, 0\n"\
      "v_mov_b32 v103, v96\n"\
      "v_mov_b32 v110, 0\n"\
      "v_mov_b32 v111, v104\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v97, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v105, -1, v[110:111]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[42:43], v51, v52\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v50, s[44:45], v50, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v88, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v90, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v66, v58\n"\
      "v_sub_co_u32_e64 v70, s[48:49], v66, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v72, v98\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v72, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v74, v106\n"\
      "v_sub_co_u32_e64 v78, s[60:61], v74, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v80, v114\n"\
      "v_sub_co_u32_e64 v84, s[66:67], v80, v114\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v82, v122\n"\
      "v_sub_co_u32_e64 v86, s[72:73], v82, v122\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v89, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v88, s[36:37], v88, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v91, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v90, s[42:43], v90, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v67, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v71, s[50:51], v67, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v73, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v73, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v75, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v79, s[62:63], v75, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v81, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v85, s[68:69], v81, v115, s[66:67]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v83, v123, s[76:77]\n"\
      "v_subb_co_u32_e64 v87, s[74:75], v83, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v89, s[38:39], v89, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v91, s[44:45], v91, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v70, s[48:49], v70, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v78, s[60:61], v78, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v84, s[66:67], v84, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v86, s[72:73], v86, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v88, s[36:37], v88, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v90, s[42:43], v90, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[14:15]\n"\
      "v_lshrrev_b32 v52, 16, v15\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[10:11]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v42, v10, v40, s[38:39]\n"\
      "v_mov_b32 v55, v48\n"\
      "v_cndmask_b32_e64 v43, v11, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v49, -1, v[54:55]\n"\
      "v_sub_co_u32_e64 v10, s[36:37], v8, v42\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_subb_co_u32_e64 v11, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v10, s[36:37], v10, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v12, v50\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v44, s[36:37]\n"\
      "v_sub_co_u32_e64 v14, s[42:43], v12, v50\n"\
      "v_lshlrev_b64 v[112:113], 28, v[30:31]\n"\
      "v_lshlrev_b64 v[120:121], 4, v[34:35]\n"\
      "v_lshrrev_b32 v116, 4, v31\n"\
      "v_lshrrev_b32 v124, 28, v35\n"\
      "v_lshrrev_b64 v[40:41], 12, v[38:39]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v13, v51, s[46:47]\n"\
      "v_lshlrev_b32 v44, 20, v38\n"\
      "v_subb_co_u32_e64 v15, s[44:45], v13, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[18:19]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_lshrrev_b32 v60, 8, v19\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v14, s[42:43], v14, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v15, s[24:25], v15, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[104:105], 12, v[26:27]\n"\
      "v_lshlrev_b64 v[48:49], 6, v[66:67]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "v_lshrrev_b64 v[96:97], 24, v[22:23]\n"\
      "v_lshrrev_b32 v108, 20, v27\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_lshrrev_b32 v52, 26, v67\n"\
      "v_lshlrev_b32 v100, 8, v22\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v36, v42\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v16, v58\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v100, 1, v[96:97]\n"\
      "v_sub_co_u32_e64 v18, s[48:49], v16, v58\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v37, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v36, s[36:37], v36, v42\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v17, v59, s[52:53]\n"\
      "v_sub_co_u32_e64 v99, s[54:55], v99, v100\n"\
      "v_subb_co_u32_e64 v19, s[50:51], v17, v59, s[48:49]\n"\
      "v_subb_co_u32_e64 v37, s[38:39], v37, v43, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v98, s[56:57], v98, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v18, s[48:49], v18, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v36, s[36:37], v36, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v24, v106\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v32, v122\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v101, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v20, v98\n"\
      "v_sub_co_u32_e64 v26, s[60:61], v24, v106\n"\
      "v_sub_co_u32_e64 v34, s[72:73], v32, v122\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v66, s[42:43], v64, v50\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v37, s[24:25], v37, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v25, v107, s[64:65]\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v28, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v33, v123, s[76:77]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v21, v99, s[58:59]\n"\
      "v_sub_co_u32_e64 v20, s[54:55], v20, v98\n"\
      "v_subb_co_u32_e64 v27, s[62:63], v25, v107, s[60:61]\n"\
      "v_sub_co_u32_e64 v30, s[66:67], v28, v114\n"\
      "v_subb_co_u32_e64 v35, s[74:75], v33, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v67, s[44:45], v65, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[56:57], 22, v[70:71]\n"\
      "v_lshlrev_b64 v[40:41], 10, v[90:91]\n"\
      "v_lshrrev_b32 v60, 10, v71\n"\
      "v_lshrrev_b32 v44, 22, v91\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v29, v115, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v21, s[56:57], v21, v99, s[54:55]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v26, s[60:61], v26, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v31, s[68:69], v29, v115, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v34, s[72:73], v34, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v66, s[42:43], v66, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v44, -1, v[40:41]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v109, 1, v[104:105]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v125, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v20, s[54:55], v20, 0, s[56:57]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v108, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v30, s[66:67], v30, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v117, 1, v[112:113]\n"\
      "v_lshrrev_b64 v[104:105], 18, v[78:79]\n"\
      "v_lshrrev_b64 v[120:121], 30, v[86:87]\n"\
      "v_lshrrev_b64 v[48:49], 6, v[94:95]\n"\
      "v_addc_co_u32_e64 v21, s[24:25], v21, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v31, s[24:25], v31, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v108, 14, v78\n"\
      "v_lshlrev_b32 v124, 2, v86\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 26, v94\n"\
      "v_lshlrev_b64 v[96:97], 30, v[74:75]\n"\
      "v_mad_u64_u32 v[106:107], s[24:25], v108, 1, v[104:105]\n"\
      "v_lshlrev_b64 v[112:113], 18, v[82:83]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v124, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v100, 2, v75\n"\
      "v_lshrrev_b32 v116, 14, v83\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_sub_co_u32_e64 v107, s[60:61], v107, v108\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_sub_co_u32_e64 v123, s[72:73], v123, v124\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[42:43], v51, v52\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v106, s[62:63], v106, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v122, s[74:75], v122, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v50, s[44:45], v50, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v109, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v76, v106\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v125, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v84, v122\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[38:39]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v92, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v68, v58\n"\
      "v_sub_co_u32_e64 v70, s[48:49], v68, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v72, v98\n"\
      "v_sub_co_u32_e64 v74, s[54:55], v72, v98\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v77, v107, s[64:65]\n"\
      "v_sub_co_u32_e64 v76, s[60:61], v76, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v80, v114\n"\
      "v_sub_co_u32_e64 v82, s[66:67], v80, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v85, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v84, s[72:73], v84, v122\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v88, v42\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v88, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v93, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v92, s[42:43], v92, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v69, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v71, s[50:51], v69, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v73, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v75, s[56:57], v73, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v77, s[62:63], v77, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v81, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v83, s[68:69], v81, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v85, s[74:75], v85, v123, s[72:73]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v89, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v89, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v93, s[44:45], v93, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v70, s[48:49], v70, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v74, s[54:55], v74, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v76, s[60:61], v76, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v82, s[66:67], v82, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v84, s[72:73], v84, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v92, s[42:43], v92, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v53, 1, v[48:49]\n"\
      "global_store_dwordx2 %[l8], v[8:9], s[78:79] offset:0\n"\
      "global_store_dwordx2 %[l8], v[10:11], s[78:79] offset:512\n"\
      "global_store_dwordx2 %[l8], v[12:13], s[78:79] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[14:15], s[78:79] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[16:17], s[78:79] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[18:19], s[78:79] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[20:21], s[78:79] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[22:23], s[78:79] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[24:25], s[80:81] offset:0\n"\
      "global_store_dwordx2 %[l8], v[26:27], s[80:81] offset:512\n"\
      "global_store_dwordx2 %[l8], v[28:29], s[80:81] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[30:31], s[80:81] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[32:33], s[80:81] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[34:35], s[80:81] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[36:37], s[80:81] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[38:39], s[80:81] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[64:65], s[82:83] offset:0\n"\
      "global_store_dwordx2 %[l8], v[66:67], s[82:83] offset:512\n"\
      "global_store_dwordx2 %[l8], v[68:69], s[82:83] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[70:71], s[82:83] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[72:73], s[82:83] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[74:75], s[82:83] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[76:77], s[82:83] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[78:79], s[82:83] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[80:81], s[84:85] offset:0\n"\
      "global_store_dwordx2 %[l8], v[82:83], s[84:85] offset:512\n"\
      "global_store_dwordx2 %[l8], v[84:85], s[84:85] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[86:87], s[84:85] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[88:89], s[84:85] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[90:91], s[84:85] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[92:93], s[84:85] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[94:95], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      :: __VA_ARGS__ \
      : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "scc", "memory")

// fwd_last: 3908 VALU, 4296 lines
#define MI_TW_BODY_FWD_LAST(...) asm volatile(\
      "s_mov_b64 s[22:23], exec\n"\
      "s_add_u32 s78, %[g_lo], 0\n"\
      "s_addc_u32 s79, %[g_hi], 0\n"\
      "s_add_u32 s80, %[g_lo], 4096\n"\
      "s_addc_u32 s81, %[g_hi], 0\n"\
      "s_add_u32 s82, %[g_lo], 8192\n"\
      "s_addc_u32 s83, %[g_hi], 0\n"\
      "s_add_u32 s84, %[g_lo], 12288\n"\
      "s_addc_u32 s85, %[g_hi], 0\n"\
      "s_add_u32 s86, %[tw_lo], 0\n"\
      "s_addc_u32 s87, %[tw_hi], 0\n"\
      "s_add_u32 s88, %[tw_lo], 4096\n"\
      "s_addc_u32 s89, %[tw_hi], 0\n"\
      "s_add_u32 s90, %[tw_lo], 8192\n"\
      "s_addc_u32 s91, %[tw_hi], 0\n"\
      "s_add_u32 s92, %[tw_lo], 12288\n"\
      "s_addc_u32 s93, %[tw_hi], 0\n"\
      "s_mov_b32 s20, 0xaaaaaaaa\n"\
      "s_mov_b32 s21, 0xaaaaaaaa\n"\
      "global_load_dwordx2 v[64:65], %[l8], s[78:79] offset:0\n"\
      "global_load_dwordx2 v[66:67], %[l8], s[78:79] offset:512\n"\
      "global_load_dwordx2 v[68:69], %[l8], s[78:79] offset:1024\n"\
      "global_load_dwordx2 v[70:71], %[l8], s[78:79] offset:1536\n"\
      "global_load_dwordx2 v[72:73], %[l8], s[78:79] offset:2048\n"\
      "global_load_dwordx2 v[74:75], %[l8], s[78:79] offset:2560\n"\
      "global_load_dwordx2 v[76:77], %[l8], s[78:79] offset:3072\n"\
      "global_load_dwordx2 v[78:79], %[l8], s[78:79] offset:3584\n"\
      "global_load_dwordx2 v[80:81], %[l8], s[80:81] offset:0\n"\
      "global_load_dwordx2 v[82:83], %[l8], s[80:81] offset:512\n"\
      "global_load_dwordx2 v[84:85], %[l8], s[80:81] offset:1024\n"\
      "global_load_dwordx2 v[86:87], %[l8], s[80:81] offset:1536\n"\
      "global_load_dwordx2 v[88:89], %[l8], s[80:81] offset:2048\n"\
      "global_load_dwordx2 v[90:91], %[l8], s[80:81] offset:2560\n"\
      "global_load_dwordx2 v[92:93], %[l8], s[80:81] offset:3072\n"\
      "global_load_dwordx2 v[94:95], %[l8], s[80:81] offset:3584\n"\
      "global_load_dwordx2 v[96:97], %[l8], s[82:83] offset:0\n"\
      "global_load_dwordx2 v[98:99], %[l8], s[82:83] offset:512\n"\
      "global_load_dwordx2 v[100:101], %[l8], s[82:83] offset:1024\n"\
      "global_load_dwordx2 v[102:103], %[l8], s[82:83] offset:1536\n"\
      "global_load_dwordx2 v[104:105], %[l8], s[82:83] offset:2048\n"\
      "global_load_dwordx2 v[106:107], %[l8], s[82:83] offset:2560\n"\
      "global_load_dwordx2 v[108:109], %[l8], s[82:83] offset:3072\n"\
      "global_load_dwordx2 v[110:111], %[l8], s[82:83] offset:3584\n"\
      "global_load_dwordx2 v[112:113], %[l8], s[84:85] offset:0\n"\
      "global_load_dwordx2 v[114:115], %[l8], s[84:85] offset:512\n"\
      "global_load_dwordx2 v[116:117], %[l8], s[84:85] offset:1024\n"\
      "global_load_dwordx2 v[118:119], %[l8], s[84:85] offset:1536\n"\
      "global_load_dwordx2 v[120:121], %[l8], s[84:85] offset:2048\n"\
      "global_load_dwordx2 v[122:123], %[l8], s[84:85] offset:2560\n"\
      "global_load_dwordx2 v[124:125], %[l8], s[84:85] offset:3072\n"\
      "global_load_dwordx2 v[126:127], %[l8], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_lshlrev_b64 v[8:9], 16, v[96:97]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[98:99]\n"\
      "v_lshrrev_b32 v12, 16, v97\n"\
      "v_lshrrev_b32 v20, 16, v99\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mov_b32 v14, 0\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v96, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v97, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v67, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v96, s[36:37], v96, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[100:101]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[102:103]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[104:105]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[106:107]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[108:109]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[110:111]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[112:113]\n"\
      "v_lshrrev_b32 v28, 16, v101\n"\
      "v_lshrrev_b32 v36, 16, v103\n"\
      "v_lshrrev_b32 v44, 16, v105\n"\
      "v_lshrrev_b32 v52, 16, v107\n"\
      "v_lshrrev_b32 v60, 16, v109\n"\
      "v_lshrrev_b32 v12, 16, v111\n"\
      "v_lshrrev_b32 v20, 16, v113\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v80, v18\n"\
      "v_sub_co_u32_e64 v100, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v102, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v104, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v106, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v108, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v110, s[36:37], v78, v10\n"\
      "v_sub_co_u32_e64 v112, s[42:43], v80, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v81, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v101, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v103, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v105, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v107, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v109, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v111, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v113, s[44:45], v81, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v100, s[48:49], v100, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v102, s[54:55], v102, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v104, s[60:61], v104, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v106, s[66:67], v106, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v108, s[72:73], v108, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v110, s[36:37], v110, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v112, s[42:43], v112, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v20, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 16, v[114:115]\n"\
      "v_lshlrev_b64 v[32:33], 16, v[116:117]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[118:119]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[120:121]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[122:123]\n"\
      "v_lshlrev_b64 v[8:9], 16, v[124:125]\n"\
      "v_lshlrev_b64 v[16:17], 16, v[126:127]\n"\
      "v_lshrrev_b32 v28, 16, v115\n"\
      "v_lshrrev_b32 v36, 16, v117\n"\
      "v_lshrrev_b32 v44, 16, v119\n"\
      "v_lshrrev_b32 v52, 16, v121\n"\
      "v_lshrrev_b32 v60, 16, v123\n"\
      "v_lshrrev_b32 v12, 16, v125\n"\
      "v_lshrrev_b32 v20, 16, v127\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v82, v26\n"\
      "v_sub_co_u32_e64 v114, s[48:49], v82, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v84, v34\n"\
      "v_sub_co_u32_e64 v116, s[54:55], v84, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v86, v42\n"\
      "v_sub_co_u32_e64 v118, s[60:61], v86, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v88, v50\n"\
      "v_sub_co_u32_e64 v120, s[66:67], v88, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v90, v58\n"\
      "v_sub_co_u32_e64 v122, s[72:73], v90, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_sub_co_u32_e64 v124, s[36:37], v92, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v94, v18\n"\
      "v_sub_co_u32_e64 v126, s[42:43], v94, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v83, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v115, s[50:51], v83, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v85, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v117, s[56:57], v85, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v87, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v119, s[62:63], v87, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v89, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v121, s[68:69], v89, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v91, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v123, s[74:75], v91, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v125, s[38:39], v93, v11, s[36:37]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v95, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v127, s[44:45], v95, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v114, s[48:49], v114, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v116, s[54:55], v116, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v118, s[60:61], v118, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v120, s[66:67], v120, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v122, s[72:73], v122, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v124, s[36:37], v124, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v126, s[42:43], v126, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v127, s[24:25], v127, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[80:81]\n"\
      "v_lshlrev_b64 v[16:17], 24, v[82:83]\n"\
      "v_lshrrev_b32 v12, 8, v81\n"\
      "v_lshrrev_b32 v20, 8, v83\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v82, s[42:43], v66, v18\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v80, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[44:45], v67, v19, s[42:43]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v82, s[42:43], v82, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v80, s[36:37], v80, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v12, s[36:37]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[112:113]\n"\
      "v_lshlrev_b32 v20, 8, v112\n"\
      "v_lshlrev_b64 v[24:25], 24, v[84:85]\n"\
      "v_lshlrev_b64 v[32:33], 24, v[86:87]\n"\
      "v_lshlrev_b64 v[40:41], 24, v[88:89]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 24, v[94:95]\n"\
      "v_lshrrev_b32 v28, 8, v85\n"\
      "v_lshrrev_b32 v36, 8, v87\n"\
      "v_lshrrev_b32 v44, 8, v89\n"\
      "v_lshrrev_b32 v52, 8, v91\n"\
      "v_lshrrev_b32 v60, 8, v93\n"\
      "v_lshrrev_b32 v12, 8, v95\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v72, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v74, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v76, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v78, v10\n"\
      "v_sub_co_u32_e64 v84, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v86, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v72, v42\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v74, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v76, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v78, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v96, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v73, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v75, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v77, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v79, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v85, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v87, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v73, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v75, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v77, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v79, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v97, s[44:45], v97, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v84, s[48:49], v84, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v86, s[54:55], v86, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v96, s[42:43], v96, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v97, s[24:25], v97, v20, s[42:43]\n"\
      "v_lshrrev_b64 v[24:25], 24, v[114:115]\n"\
      "v_lshrrev_b64 v[32:33], 24, v[116:117]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[118:119]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 24, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 24, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 24, v[126:127]\n"\
      "v_lshlrev_b32 v28, 8, v114\n"\
      "v_lshlrev_b32 v36, 8, v116\n"\
      "v_lshlrev_b32 v44, 8, v118\n"\
      "v_lshlrev_b32 v52, 8, v120\n"\
      "v_lshlrev_b32 v60, 8, v122\n"\
      "v_lshlrev_b32 v12, 8, v124\n"\
      "v_lshlrev_b32 v20, 8, v126\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v28, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_sub_co_u32_e64 v27, s[48:49], v27, v28\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[48:49]\n"\
      "v_addc_co_u32_e64 v26, s[50:51], v26, 0, s[48:49]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v29, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v104, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v106, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v108, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v110, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_sub_co_u32_e64 v98, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v100, s[54:55], v100, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v102, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v105, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v104, s[66:67], v104, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v107, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v106, s[72:73], v106, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v109, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v108, s[36:37], v108, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v111, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v110, s[42:43], v110, v18\n"\
      "v_subb_co_u32_e64 v99, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v101, s[56:57], v101, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v103, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v105, s[68:69], v105, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v107, s[74:75], v107, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v109, s[38:39], v109, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v111, s[44:45], v111, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v98, s[48:49], v98, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v100, s[54:55], v100, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v102, s[60:61], v102, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v104, s[66:67], v104, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v106, s[72:73], v106, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v108, s[36:37], v108, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v110, s[42:43], v110, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[116:117], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 12, v[72:73]\n"\
      "v_lshlrev_b64 v[16:17], 12, v[74:75]\n"\
      "v_lshrrev_b32 v12, 20, v73\n"\
      "v_lshrrev_b32 v20, 20, v75\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_sub_co_u32_e64 v72, s[36:37], v64, v10\n"\
      "v_sub_co_u32_e64 v74, s[42:43], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v73, s[38:39], v65, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v75, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 28, v[88:89]\n"\
      "v_lshrrev_b32 v44, 4, v89\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v72, s[36:37], v72, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v74, s[42:43], v74, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshlrev_b64 v[48:49], 28, v[90:91]\n"\
      "v_lshlrev_b64 v[56:57], 28, v[92:93]\n"\
      "v_lshlrev_b64 v[8:9], 28, v[94:95]\n"\
      "v_lshlrev_b64 v[16:17], 4, v[104:105]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshrrev_b32 v52, 4, v91\n"\
      "v_lshrrev_b32 v60, 4, v93\n"\
      "v_lshrrev_b32 v12, 4, v95\n"\
      "v_lshrrev_b32 v20, 28, v105\n"\
      "v_lshlrev_b64 v[24:25], 12, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 12, v[78:79]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 20, v77\n"\
      "v_lshrrev_b32 v36, 20, v79\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v68, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v70, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v68, v26\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v70, v34\n"\
      "v_sub_co_u32_e64 v88, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v69, v27, s[52:53]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v71, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v69, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v71, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v89, s[62:63], v81, v43, s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v88, s[60:61], v88, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v84, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v86, v10\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[66:67], v82, v50\n"\
      "v_sub_co_u32_e64 v92, s[72:73], v84, v58\n"\
      "v_sub_co_u32_e64 v94, s[36:37], v86, v10\n"\
      "v_sub_co_u32_e64 v104, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v85, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v87, v11, s[40:41]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v91, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v93, s[74:75], v85, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v95, s[38:39], v87, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v105, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 4, v[106:107]\n"\
      "v_lshlrev_b64 v[32:33], 4, v[108:109]\n"\
      "v_lshlrev_b64 v[40:41], 4, v[110:111]\n"\
      "v_lshrrev_b32 v28, 28, v107\n"\
      "v_lshrrev_b32 v36, 28, v109\n"\
      "v_lshrrev_b32 v44, 28, v111\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v90, s[66:67], v90, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v92, s[72:73], v92, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v94, s[36:37], v94, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v104, s[42:43], v104, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[60:61]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[120:121]\n"\
      "v_lshrrev_b64 v[56:57], 12, v[122:123]\n"\
      "v_lshrrev_b64 v[8:9], 12, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 12, v[126:127]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 20, v120\n"\
      "v_lshlrev_b32 v60, 20, v122\n"\
      "v_lshlrev_b32 v12, 20, v124\n"\
      "v_lshlrev_b32 v20, 20, v126\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[66:67], v51, v52\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v50, s[68:69], v50, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v116, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v118, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v106, s[48:49], v98, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v100, v34\n"\
      "v_sub_co_u32_e64 v108, s[54:55], v100, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v102, v42\n"\
      "v_sub_co_u32_e64 v110, s[60:61], v102, v42\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_sub_co_u32_e64 v112, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v114, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v117, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v116, s[36:37], v116, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v119, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v118, s[42:43], v118, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v107, s[50:51], v99, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v101, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v109, s[56:57], v101, v35, s[54:55]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v103, v43, s[64:65]\n"\
      "v_subb_co_u32_e64 v111, s[62:63], v103, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v113, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v115, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v117, s[38:39], v117, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v119, s[44:45], v119, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v106, s[48:49], v106, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v108, s[54:55], v108, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v110, s[60:61], v110, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v112, s[66:67], v112, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v114, s[72:73], v114, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v116, s[36:37], v116, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v118, s[42:43], v118, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v111, s[24:25], v111, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v113, s[24:25], v113, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[8:9], 6, v[68:69]\n"\
      "v_lshrrev_b32 v12, 26, v69\n"\
      "v_lshlrev_b64 v[16:17], 6, v[70:71]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 26, v71\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_lshlrev_b64 v[24:25], 22, v[76:77]\n"\
      "v_lshlrev_b64 v[32:33], 22, v[78:79]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshrrev_b32 v28, 10, v77\n"\
      "v_lshrrev_b32 v36, 10, v79\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_sub_co_u32_e64 v68, s[36:37], v64, v10\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v66, v18\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v66, v18\n"\
      "v_subb_co_u32_e64 v69, s[38:39], v65, v11, s[36:37]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshrrev_b64 v[56:57], 18, v[92:93]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v67, v19, s[46:47]\n"\
      "v_lshlrev_b32 v60, 14, v92\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v67, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[40:41], 30, v[84:85]\n"\
      "v_lshlrev_b64 v[48:49], 30, v[86:87]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v68, s[36:37], v68, 0, s[38:39]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v44, 2, v85\n"\
      "v_lshrrev_b32 v52, 2, v87\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_lshrrev_b64 v[8:9], 18, v[94:95]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_lshlrev_b32 v12, 14, v94\n"\
      "v_lshlrev_b64 v[16:17], 18, v[100:101]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_lshrrev_b32 v20, 14, v101\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v82, v50\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v82, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v88, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v83, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v83, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v89, s[74:75], v89, v59, s[72:73]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v90, v10\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v88, s[72:73], v88, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v74, v34\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_sub_co_u32_e64 v78, s[54:55], v74, v34\n"\
      "v_sub_co_u32_e64 v84, s[60:61], v80, v42\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v91, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v90, v10\n"\
      "v_sub_co_u32_e64 v100, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v60, s[72:73]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v75, v35, s[58:59]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v76, s[48:49], v72, v26\n"\
      "v_subb_co_u32_e64 v79, s[56:57], v75, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v85, s[62:63], v81, v43, s[60:61]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v91, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v101, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 10, v[116:117]\n"\
      "v_lshlrev_b64 v[56:57], 10, v[118:119]\n"\
      "v_lshrrev_b32 v52, 22, v117\n"\
      "v_lshrrev_b32 v60, 22, v119\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v77, s[50:51], v73, v27, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v78, s[54:55], v78, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v84, s[60:61], v84, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v100, s[42:43], v100, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v37, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v76, s[48:49], v76, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[60:61]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v101, s[24:25], v101, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_lshrrev_b64 v[32:33], 30, v[108:109]\n"\
      "v_lshrrev_b64 v[40:41], 30, v[110:111]\n"\
      "v_lshrrev_b64 v[8:9], 6, v[124:125]\n"\
      "v_lshrrev_b64 v[16:17], 6, v[126:127]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v28, s[48:49]\n"\
      "v_lshlrev_b32 v36, 2, v108\n"\
      "v_lshlrev_b32 v44, 2, v110\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v12, 26, v124\n"\
      "v_lshlrev_b32 v20, 26, v126\n"\
      "v_lshlrev_b64 v[24:25], 18, v[102:103]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_lshrrev_b32 v28, 14, v103\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v106, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v122, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v98, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v98, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v104, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v107, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v106, s[60:61], v106, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v116, s[66:67], v112, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v114, v58\n"\
      "v_sub_co_u32_e64 v118, s[72:73], v114, v58\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v120, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v123, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v122, s[42:43], v122, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v99, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v99, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v105, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v107, s[62:63], v107, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v117, s[68:69], v113, v51, s[66:67]\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v115, v59, s[76:77]\n"\
      "v_subb_co_u32_e64 v119, s[74:75], v115, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v121, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v123, s[44:45], v123, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v104, s[54:55], v104, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v106, s[60:61], v106, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v116, s[66:67], v116, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v118, s[72:73], v118, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v120, s[36:37], v120, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v122, s[42:43], v122, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v105, s[24:25], v105, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v119, s[24:25], v119, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v121, s[24:25], v121, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[124:125], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "v_lshlrev_b64 v[16:17], 19, v[70:71]\n"\
      "v_lshlrev_b64 v[8:9], 3, v[66:67]\n"\
      "v_lshrrev_b32 v20, 13, v71\n"\
      "v_lshrrev_b32 v12, 29, v67\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v20, 1, v[18:19]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_mov_b32 v22, 0\n"\
      "v_mov_b32 v23, v16\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v64, v10\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v17, -1, v[22:23]\n"\
      "v_sub_co_u32_e64 v66, s[36:37], v64, v10\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v65, v11, s[40:41]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_subb_co_u32_e64 v67, s[38:39], v65, v11, s[36:37]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v66, s[36:37], v66, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v13, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v68, v18\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v12, s[36:37]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v68, v18\n"\
      "v_lshlrev_b64 v[48:49], 31, v[86:87]\n"\
      "v_lshlrev_b64 v[56:57], 7, v[90:91]\n"\
      "v_lshrrev_b64 v[32:33], 21, v[78:79]\n"\
      "v_lshrrev_b32 v52, 1, v87\n"\
      "v_lshrrev_b32 v60, 25, v91\n"\
      "v_lshrrev_b64 v[8:9], 9, v[94:95]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v69, v19, s[46:47]\n"\
      "v_lshlrev_b32 v36, 11, v78\n"\
      "v_lshlrev_b32 v12, 23, v94\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v69, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 27, v[74:75]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v60, -1, v[56:57]\n"\
      "v_lshrrev_b32 v28, 5, v75\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v36, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v12, 1, v[8:9]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v35, s[54:55], v35, v36\n"\
      "v_sub_co_u32_e64 v11, s[36:37], v11, v12\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v34, s[56:57], v34, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v10, s[38:39], v10, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 15, v[82:83]\n"\
      "v_lshlrev_b64 v[16:17], 9, v[98:99]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "v_lshrrev_b32 v44, 17, v83\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v20, 23, v99\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v37, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v76, v34\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v13, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v92, v10\n"\
      "v_mad_u64_u32 v[42:43], s[60:61], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[58:59], s[72:73], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[18:19], s[42:43], v20, -1, v[16:17]\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v72, v26\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v72, v26\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v77, v35, s[58:59]\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v76, v34\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v93, v11, s[40:41]\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v92, v10\n"\
      "v_mad_u64_u32 v[40:41], s[62:63], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[74:75], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[16:17], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v73, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v73, v27, s[48:49]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v77, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v93, v11, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v16, s[44:45]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v80, v42\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v88, v58\n"\
      "v_cndmask_b32_e64 v19, v19, v17, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v96, v18\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v29, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v37, 1, v[32:33]\n"\
      "v_sub_co_u32_e64 v82, s[60:61], v80, v42\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v88, v58\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v13, 1, v[8:9]\n"\
      "v_sub_co_u32_e64 v98, s[42:43], v96, v18\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v28, s[48:49]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v36, s[54:55]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v12, s[36:37]\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v81, v43, s[64:65]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v84, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v89, v59, s[76:77]\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v97, v19, s[46:47]\n"\
      "v_subb_co_u32_e64 v83, s[62:63], v81, v43, s[60:61]\n"\
      "v_sub_co_u32_e64 v86, s[66:67], v84, v50\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v89, v59, s[72:73]\n"\
      "v_subb_co_u32_e64 v99, s[44:45], v97, v19, s[42:43]\n"\
      "v_lshlrev_b64 v[24:25], 25, v[102:103]\n"\
      "v_lshlrev_b64 v[32:33], 1, v[106:107]\n"\
      "v_lshlrev_b64 v[8:9], 13, v[122:123]\n"\
      "v_lshrrev_b32 v28, 7, v103\n"\
      "v_lshrrev_b32 v36, 31, v107\n"\
      "v_lshrrev_b32 v12, 19, v123\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v85, v51, s[70:71]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v82, s[60:61], v82, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v87, s[68:69], v85, v51, s[66:67]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v98, s[42:43], v98, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v28, -1, v[24:25]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v36, -1, v[32:33]\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v12, -1, v[8:9]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v21, 1, v[16:17]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v44, s[60:61]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v86, s[66:67], v86, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v60, s[72:73]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v20, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[84:85], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshrrev_b64 v[40:41], 15, v[110:111]\n"\
      "v_lshrrev_b64 v[56:57], 27, v[118:119]\n"\
      "v_lshrrev_b64 v[16:17], 3, v[126:127]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v28, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v36, 1, v[34:35]\n"\
      "v_lshlrev_b32 v44, 17, v110\n"\
      "v_lshlrev_b32 v60, 5, v118\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v12, 1, v[10:11]\n"\
      "v_lshlrev_b32 v20, 29, v126\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshlrev_b64 v[48:49], 21, v[114:115]\n"\
      "v_mad_u64_u32 v[58:59], s[24:25], v60, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v20, 1, v[16:17]\n"\
      "v_mov_b32 v30, 0\n"\
      "v_mov_b32 v31, v24\n"\
      "v_mov_b32 v38, 0\n"\
      "v_mov_b32 v39, v32\n"\
      "v_lshrrev_b32 v52, 11, v115\n"\
      "v_mov_b32 v14, 0\n"\
      "v_mov_b32 v15, v8\n"\
      "v_mad_u64_u32 v[26:27], s[48:49], v25, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[34:35], s[54:55], v33, -1, v[38:39]\n"\
      "v_sub_co_u32_e64 v43, s[60:61], v43, v44\n"\
      "v_mad_u64_u32 v[50:51], s[66:67], v52, -1, v[48:49]\n"\
      "v_sub_co_u32_e64 v59, s[72:73], v59, v60\n"\
      "v_mad_u64_u32 v[10:11], s[36:37], v9, -1, v[14:15]\n"\
      "v_sub_co_u32_e64 v19, s[42:43], v19, v20\n"\
      "v_mad_u64_u32 v[24:25], s[50:51], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[32:33], s[56:57], -1, 1, v[34:35]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v42, s[62:63], v42, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[48:49], s[68:69], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v58, s[74:75], v58, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[8:9], s[38:39], -1, 1, v[10:11]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v18, s[44:45], v18, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v26, v26, v24, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v34, v34, v32, s[56:57]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[62:63]\n"\
      "v_add_co_u32_e64 v40, s[64:65], v108, v42\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[68:69]\n"\
      "v_addc_co_u32_e64 v59, s[24:25], v59, v61, s[74:75]\n"\
      "v_add_co_u32_e64 v56, s[76:77], v116, v58\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v10, v10, v8, s[38:39]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v21, s[44:45]\n"\
      "v_add_co_u32_e64 v16, s[46:47], v124, v18\n"\
      "v_cndmask_b32_e64 v27, v27, v25, s[50:51]\n"\
      "v_add_co_u32_e64 v24, s[52:53], v100, v26\n"\
      "v_sub_co_u32_e64 v102, s[48:49], v100, v26\n"\
      "v_cndmask_b32_e64 v35, v35, v33, s[56:57]\n"\
      "v_add_co_u32_e64 v32, s[58:59], v104, v34\n"\
      "v_sub_co_u32_e64 v106, s[54:55], v104, v34\n"\
      "v_addc_co_u32_e64 v41, s[64:65], v109, v43, s[64:65]\n"\
      "v_sub_co_u32_e64 v108, s[60:61], v108, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[68:69]\n"\
      "v_add_co_u32_e64 v48, s[70:71], v112, v50\n"\
      "v_sub_co_u32_e64 v114, s[66:67], v112, v50\n"\
      "v_addc_co_u32_e64 v57, s[76:77], v117, v59, s[76:77]\n"\
      "v_sub_co_u32_e64 v116, s[72:73], v116, v58\n"\
      "v_cndmask_b32_e64 v11, v11, v9, s[38:39]\n"\
      "v_add_co_u32_e64 v8, s[40:41], v120, v10\n"\
      "v_sub_co_u32_e64 v122, s[36:37], v120, v10\n"\
      "v_addc_co_u32_e64 v17, s[46:47], v125, v19, s[46:47]\n"\
      "v_sub_co_u32_e64 v124, s[42:43], v124, v18\n"\
      "v_addc_co_u32_e64 v25, s[52:53], v101, v27, s[52:53]\n"\
      "v_subb_co_u32_e64 v103, s[50:51], v101, v27, s[48:49]\n"\
      "v_addc_co_u32_e64 v33, s[58:59], v105, v35, s[58:59]\n"\
      "v_subb_co_u32_e64 v107, s[56:57], v105, v35, s[54:55]\n"\
      "v_subb_co_u32_e64 v109, s[62:63], v109, v43, s[60:61]\n"\
      "v_addc_co_u32_e64 v49, s[70:71], v113, v51, s[70:71]\n"\
      "v_subb_co_u32_e64 v115, s[68:69], v113, v51, s[66:67]\n"\
      "v_subb_co_u32_e64 v117, s[74:75], v117, v59, s[72:73]\n"\
      "v_addc_co_u32_e64 v9, s[40:41], v121, v11, s[40:41]\n"\
      "v_subb_co_u32_e64 v123, s[38:39], v121, v11, s[36:37]\n"\
      "v_subb_co_u32_e64 v125, s[44:45], v125, v19, s[42:43]\n"\
      "v_cndmask_b32_e64 v28, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v102, s[48:49], v102, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v29, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v36, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v106, s[54:55], v106, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v37, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v108, s[60:61], v108, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v114, s[66:67], v114, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v116, s[72:73], v116, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v12, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v122, s[36:37], v122, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v20, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v124, s[42:43], v124, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v21, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v103, s[24:25], v103, v28, s[48:49]\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v29, 1, v[24:25]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v36, s[54:55]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v37, 1, v[32:33]\n"\
      "v_addc_co_u32_e64 v109, s[24:25], v109, v44, s[60:61]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v52, s[66:67]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v117, s[24:25], v117, v60, s[72:73]\n"\
      "v_mad_u64_u32 v[118:119], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v12, s[36:37]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v13, 1, v[8:9]\n"\
      "v_addc_co_u32_e64 v125, s[24:25], v125, v20, s[42:43]\n"\
      "v_mad_u64_u32 v[126:127], s[24:25], v21, 1, v[16:17]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[86:87] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[86:87] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[86:87] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[86:87] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[86:87] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[86:87] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[86:87] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[86:87] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v64, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v66, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v64, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v66, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v65, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v65, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v67, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v67, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v68, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v64, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v65, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v66, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v67, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v70, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v72, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v68, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v70, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v72, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v69, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v69, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v71, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v71, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v73, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v73, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v68, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v69, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v70, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v71, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v72, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v73, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v74, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v76, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v78, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v74, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v76, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v78, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v75, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v75, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v77, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v77, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v79, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v79, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v74, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v75, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v76, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v77, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v78, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v79, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[88:89] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[88:89] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[88:89] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[88:89] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[88:89] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[88:89] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[88:89] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[88:89] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v80, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v82, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v80, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v82, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v81, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v81, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v83, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v83, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v84, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v80, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v81, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v82, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v83, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v86, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v88, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v84, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v86, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v88, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v85, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v85, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v87, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v87, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v89, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v89, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v84, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v85, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v86, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v87, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v88, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v89, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v90, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v92, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v94, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v90, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v92, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v94, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v91, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v91, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v93, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v93, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v95, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v95, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v90, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v91, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v92, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v93, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v94, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v95, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[90:91] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[90:91] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[90:91] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[90:91] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[90:91] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[90:91] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[90:91] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[90:91] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v96, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v98, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v96, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v98, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v97, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v97, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v99, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v99, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v100, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v96, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v97, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v98, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v99, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v102, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v104, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v100, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v102, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v104, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v101, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v101, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v103, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v103, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v105, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v105, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v100, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v101, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v102, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v103, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v104, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v106, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v108, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v110, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v106, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v108, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v110, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v107, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v107, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v109, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v109, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v111, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v111, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v106, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v107, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v108, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v109, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v110, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v111, v37, v41, s[44:45]\n"\
      "global_load_dwordx2 v[8:9], %[l8], s[92:93] offset:0\n"\
      "global_load_dwordx2 v[10:11], %[l8], s[92:93] offset:512\n"\
      "global_load_dwordx2 v[12:13], %[l8], s[92:93] offset:1024\n"\
      "global_load_dwordx2 v[14:15], %[l8], s[92:93] offset:1536\n"\
      "global_load_dwordx2 v[16:17], %[l8], s[92:93] offset:2048\n"\
      "global_load_dwordx2 v[18:19], %[l8], s[92:93] offset:2560\n"\
      "global_load_dwordx2 v[20:21], %[l8], s[92:93] offset:3072\n"\
      "global_load_dwordx2 v[22:23], %[l8], s[92:93] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v112, v8, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v114, v10, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v112, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v114, v11, v[44:45]\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v113, v8, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v113, v9, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v115, v10, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v115, v11, v[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v116, v12, 0\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_mov_b32 v57, 0\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_mov_b32 v56, v49\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v112, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v113, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v114, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v115, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v118, v14, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v120, v16, 0\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v116, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v118, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v120, v17, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v117, v12, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v117, v13, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v119, v14, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v119, v15, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v121, v16, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v121, v17, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v116, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v117, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v118, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v119, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v120, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v121, v37, v41, s[44:45]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v122, v18, 0\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v124, v20, 0\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v126, v22, 0\n"\
      "v_mov_b32 v57, 0\n"\
      "v_mov_b32 v56, v49\n"\
      "v_mov_b32 v33, 0\n"\
      "v_mov_b32 v32, v25\n"\
      "v_mov_b32 v45, 0\n"\
      "v_mov_b32 v44, v37\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v122, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v124, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v126, v23, v[44:45]\n"\
      "v_mov_b32 v59, 0\n"\
      "v_mov_b32 v58, v50\n"\
      "v_mov_b32 v56, v51\n"\
      "v_mov_b32 v35, 0\n"\
      "v_mov_b32 v34, v26\n"\
      "v_mov_b32 v32, v27\n"\
      "v_mov_b32 v47, 0\n"\
      "v_mov_b32 v46, v38\n"\
      "v_mov_b32 v44, v39\n"\
      "v_mad_u64_u32 v[52:53], s[24:25], v123, v18, v[58:59]\n"\
      "v_mad_u64_u32 v[54:55], s[24:25], v123, v19, v[56:57]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v125, v20, v[34:35]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v125, v21, v[32:33]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v127, v22, v[46:47]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v127, v23, v[44:45]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v53, 1, v[54:55]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v29, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v41, 1, v[42:43]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v48, v51\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v24, v27\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v36, v39\n"\
      "v_subb_co_u32_e64 v55, s[50:51], v52, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[38:39], v28, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[44:45], v40, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, 0, -1, s[50:51]\n"\
      "v_cndmask_b32_e64 v34, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v46, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v54, s[48:49], v54, v58\n"\
      "v_sub_co_u32_e64 v30, s[36:37], v30, v34\n"\
      "v_sub_co_u32_e64 v42, s[42:43], v42, v46\n"\
      "v_subb_co_u32_e64 v55, s[24:25], v55, 0, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[24:25], v31, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v43, s[24:25], v43, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[48:49], v50, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[24:25], s[36:37], v26, -1, v[30:31]\n"\
      "v_mad_u64_u32 v[36:37], s[42:43], v38, -1, v[42:43]\n"\
      "v_mad_u64_u32 v[52:53], s[50:51], -1, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[28:29], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[40:41], s[44:45], -1, 1, v[36:37]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v122, v48, v52, s[50:51]\n"\
      "v_cndmask_b32_e64 v123, v49, v53, s[50:51]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v124, v24, v28, s[38:39]\n"\
      "v_cndmask_b32_e64 v125, v25, v29, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v126, v36, v40, s[44:45]\n"\
      "v_cndmask_b32_e64 v127, v37, v41, s[44:45]\n"\
      "s_mov_b32 exec_lo, -1\n"\
      "s_mov_b32 exec_hi, 0\n"\
      "ds_write_b64 %[t1w], v[64:65] offset:0\n"\
      "ds_write_b64 %[t1w], v[66:67] offset:272\n"\
      "ds_write_b64 %[t1w], v[68:69] offset:544\n"\
      "ds_write_b64 %[t1w], v[70:71] offset:816\n"\
      "ds_write_b64 %[t1w], v[72:73] offset:1088\n"\
      "ds_write_b64 %[t1w], v[74:75] offset:1360\n"\
      "ds_write_b64 %[t1w], v[76:77] offset:1632\n"\
      "ds_write_b64 %[t1w], v[78:79] offset:1904\n"\
      "ds_write_b64 %[t1w], v[80:81] offset:2176\n"\
      "ds_write_b64 %[t1w], v[82:83] offset:2448\n"\
      "ds_write_b64 %[t1w], v[84:85] offset:2720\n"\
      "ds_write_b64 %[t1w], v[86:87] offset:2992\n"\
      "ds_write_b64 %[t1w], v[88:89] offset:3264\n"\
      "ds_write_b64 %[t1w], v[90:91] offset:3536\n"\
      "ds_write_b64 %[t1w], v[92:93] offset:3808\n"\
      "ds_write_b64 %[t1w], v[94:95] offset:4080\n"\
      "ds_write_b64 %[t1w], v[96:97] offset:4352\n"\
      "ds_write_b64 %[t1w], v[98:99] offset:4624\n"\
      "ds_write_b64 %[t1w], v[100:101] offset:4896\n"\
      "ds_write_b64 %[t1w], v[102:103] offset:5168\n"\
      "ds_write_b64 %[t1w], v[104:105] offset:5440\n"\
      "ds_write_b64 %[t1w], v[106:107] offset:5712\n"\
      "ds_write_b64 %[t1w], v[108:109] offset:5984\n"\
      "ds_write_b64 %[t1w], v[110:111] offset:6256\n"\
      "ds_write_b64 %[t1w], v[112:113] offset:6528\n"\
      "ds_write_b64 %[t1w], v[114:115] offset:6800\n"\
      "ds_write_b64 %[t1w], v[116:117] offset:7072\n"\
      "ds_write_b64 %[t1w], v[118:119] offset:7344\n"\
      "ds_write_b64 %[t1w], v[120:121] offset:7616\n"\
      "ds_write_b64 %[t1w], v[122:123] offset:7888\n"\
      "ds_write_b64 %[t1w], v[124:125] offset:8160\n"\
      "ds_write_b64 %[t1w], v[126:127] offset:8432\n"\
      "s_mov_b64 exec, s[22:23]\n"\
      "ds_read_b64 v[8:9], %[t1r] offset:0\n"\
      "ds_read_b64 v[10:11], %[t1r] offset:16\n"\
      "ds_read_b64 v[12:13], %[t1r] offset:32\n"\
      "ds_read_b64 v[14:15], %[t1r] offset:48\n"\
      "ds_read_b64 v[16:17], %[t1r] offset:64\n"\
      "ds_read_b64 v[18:19], %[t1r] offset:80\n"\
      "ds_read_b64 v[20:21], %[t1r] offset:96\n"\
      "ds_read_b64 v[22:23], %[t1r] offset:112\n"\
      "ds_read_b64 v[24:25], %[t1r] offset:128\n"\
      "ds_read_b64 v[26:27], %[t1r] offset:144\n"\
      "ds_read_b64 v[28:29], %[t1r] offset:160\n"\
      "ds_read_b64 v[30:31], %[t1r] offset:176\n"\
      "ds_read_b64 v[32:33], %[t1r] offset:192\n"\
      "ds_read_b64 v[34:35], %[t1r] offset:208\n"\
      "ds_read_b64 v[36:37], %[t1r] offset:224\n"\
      "ds_read_b64 v[38:39], %[t1r] offset:240\n"\
      "s_mov_b32 exec_lo, 0\n"\
      "s_mov_b32 exec_hi, -1\n"\
      "ds_write_b64 %[t1w], v[64:65] offset:0\n"\
      "ds_write_b64 %[t1w], v[66:67] offset:272\n"\
      "ds_write_b64 %[t1w], v[68:69] offset:544\n"\
      "ds_write_b64 %[t1w], v[70:71] offset:816\n"\
      "ds_write_b64 %[t1w], v[72:73] offset:1088\n"\
      "ds_write_b64 %[t1w], v[74:75] offset:1360\n"\
      "ds_write_b64 %[t1w], v[76:77] offset:1632\n"\
      "ds_write_b64 %[t1w], v[78:79] offset:1904\n"\
      "ds_write_b64 %[t1w], v[80:81] offset:2176\n"\
      "ds_write_b64 %[t1w], v[82:83] offset:2448\n"\
      "ds_write_b64 %[t1w], v[84:85] offset:2720\n"\
      "ds_write_b64 %[t1w], v[86:87] offset:2992\n"\
      "ds_write_b64 %[t1w], v[88:89] offset:3264\n"\
      "ds_write_b64 %[t1w], v[90:91] offset:3536\n"\
      "ds_write_b64 %[t1w], v[92:93] offset:3808\n"\
      "ds_write_b64 %[t1w], v[94:95] offset:4080\n"\
      "ds_write_b64 %[t1w], v[96:97] offset:4352\n"\
      "ds_write_b64 %[t1w], v[98:99] offset:4624\n"\
      "ds_write_b64 %[t1w], v[100:101] offset:4896\n"\
      "ds_write_b64 %[t1w], v[102:103] offset:5168\n"\
      "ds_write_b64 %[t1w], v[104:105] offset:5440\n"\
      "ds_write_b64 %[t1w], v[106:107] offset:5712\n"\
      "ds_write_b64 %[t1w], v[108:109] offset:5984\n"\
      "ds_write_b64 %[t1w], v[110:111] offset:6256\n"\
      "ds_write_b64 %[t1w], v[112:113] offset:6528\n"\
      "ds_write_b64 %[t1w], v[114:115] offset:6800\n"\
      "ds_write_b64 %[t1w], v[116:117] offset:7072\n"\
      "ds_write_b64 %[t1w], v[118:119] offset:7344\n"\
      "ds_write_b64 %[t1w], v[120:121] offset:7616\n"\
      "ds_write_b64 %[t1w], v[122:123] offset:7888\n"\
      "ds_write_b64 %[t1w], v[124:125] offset:8160\n"\
      "ds_write_b64 %[t1w], v[126:127] offset:8432\n"\
      "s_mov_b64 exec, s[22:23]\n"\
      "s_waitcnt lgkmcnt(0)\n"\
      "ds_read_b64 v[64:65], %[t1r] offset:0\n"\
      "ds_read_b64 v[66:67], %[t1r] offset:16\n"\
      "ds_read_b64 v[68:69], %[t1r] offset:32\n"\
      "ds_read_b64 v[70:71], %[t1r] offset:48\n"\
      "ds_read_b64 v[72:73], %[t1r] offset:64\n"\
      "ds_read_b64 v[74:75], %[t1r] offset:80\n"\
      "ds_read_b64 v[76:77], %[t1r] offset:96\n"\
      "ds_read_b64 v[78:79], %[t1r] offset:112\n"\
      "ds_read_b64 v[80:81], %[t1r] offset:128\n"\
      "ds_read_b64 v[82:83], %[t1r] offset:144\n"\
      "ds_read_b64 v[84:85], %[t1r] offset:160\n"\
      "ds_read_b64 v[86:87], %[t1r] offset:176\n"\
      "ds_read_b64 v[88:89], %[t1r] offset:192\n"\
      "ds_read_b64 v[90:91], %[t1r] offset:208\n"\
      "ds_read_b64 v[92:93], %[t1r] offset:224\n"\
      "ds_read_b64 v[94:95], %[t1r] offset:240\n"\
      "s_waitcnt lgkmcnt(0)\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[64:65]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[66:67]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[68:69]\n"\
      "v_cndmask_b32_e64 v42, v64, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v50, v66, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v43, v65, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_cndmask_b32_e64 v51, v67, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v64, s[36:37], v8, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v66, s[42:43], v10, v50\n"\
      "v_subb_co_u32_e64 v65, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v67, s[44:45], v11, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v64, s[36:37], v64, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v66, s[42:43], v66, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[70:71]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[72:73]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[74:75]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[76:77]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[78:79]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[80:81]\n"\
      "v_cndmask_b32_e64 v58, v68, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v70, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v72, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v114, v74, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v122, v76, v120, s[74:75]\n"\
      "v_cndmask_b32_e64 v42, v78, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v50, v80, v48, s[44:45]\n"\
      "v_addc_co_u32_e64 v65, s[24:25], v65, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v59, v69, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v12, v58\n"\
      "v_cndmask_b32_e64 v99, v71, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v14, v98\n"\
      "v_cndmask_b32_e64 v107, v73, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v16, v106\n"\
      "v_cndmask_b32_e64 v115, v75, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v18, v114\n"\
      "v_cndmask_b32_e64 v123, v77, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v20, v122\n"\
      "v_cndmask_b32_e64 v43, v79, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v22, v42\n"\
      "v_cndmask_b32_e64 v51, v81, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v24, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v13, v59, s[52:53]\n"\
      "v_sub_co_u32_e64 v68, s[48:49], v12, v58\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v15, v99, s[58:59]\n"\
      "v_sub_co_u32_e64 v70, s[54:55], v14, v98\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v17, v107, s[64:65]\n"\
      "v_sub_co_u32_e64 v72, s[60:61], v16, v106\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v19, v115, s[70:71]\n"\
      "v_sub_co_u32_e64 v74, s[66:67], v18, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v21, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v76, s[72:73], v20, v122\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v23, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v78, s[36:37], v22, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v25, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v80, s[42:43], v24, v50\n"\
      "v_subb_co_u32_e64 v69, s[50:51], v13, v59, s[48:49]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_subb_co_u32_e64 v71, s[56:57], v15, v99, s[54:55]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_subb_co_u32_e64 v73, s[62:63], v17, v107, s[60:61]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_subb_co_u32_e64 v75, s[68:69], v19, v115, s[66:67]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_subb_co_u32_e64 v77, s[74:75], v21, v123, s[72:73]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_subb_co_u32_e64 v79, s[38:39], v23, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v81, s[44:45], v25, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v68, s[48:49], v68, 0, s[50:51]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v61, 1, v[56:57]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v70, s[54:55], v70, 0, s[56:57]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v72, s[60:61], v72, 0, s[62:63]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v109, 1, v[104:105]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v74, s[66:67], v74, 0, s[68:69]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v117, 1, v[112:113]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v76, s[72:73], v76, 0, s[74:75]\n"\
      "v_mad_u64_u32 v[20:21], s[24:25], v125, 1, v[120:121]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v78, s[36:37], v78, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v80, s[42:43], v80, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[82:83]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[84:85]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[86:87]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[88:89]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[90:91]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[92:93]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[94:95]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v108, s[60:61]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v58, v82, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v84, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v86, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v114, v88, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v122, v90, v120, s[74:75]\n"\
      "v_cndmask_b32_e64 v42, v92, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v50, v94, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v59, v83, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v26, v58\n"\
      "v_sub_co_u32_e64 v82, s[48:49], v26, v58\n"\
      "v_cndmask_b32_e64 v99, v85, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v28, v98\n"\
      "v_sub_co_u32_e64 v84, s[54:55], v28, v98\n"\
      "v_cndmask_b32_e64 v107, v87, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v30, v106\n"\
      "v_sub_co_u32_e64 v86, s[60:61], v30, v106\n"\
      "v_cndmask_b32_e64 v115, v89, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v32, v114\n"\
      "v_sub_co_u32_e64 v88, s[66:67], v32, v114\n"\
      "v_cndmask_b32_e64 v123, v91, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v34, v122\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v34, v122\n"\
      "v_cndmask_b32_e64 v43, v93, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v36, v42\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v36, v42\n"\
      "v_cndmask_b32_e64 v51, v95, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v38, v50\n"\
      "v_sub_co_u32_e64 v94, s[42:43], v38, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v27, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v83, s[50:51], v27, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v29, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v85, s[56:57], v29, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v31, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v87, s[62:63], v31, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v33, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v89, s[68:69], v33, v115, s[66:67]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v35, v123, s[76:77]\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v35, v123, s[72:73]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v37, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v37, v43, s[36:37]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v39, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v95, s[44:45], v39, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v82, s[48:49], v82, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v84, s[54:55], v84, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v86, s[60:61], v86, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v88, s[66:67], v88, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v94, s[42:43], v94, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[26:27]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[24:25]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_cndmask_b32_e64 v50, v26, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v51, v27, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_sub_co_u32_e64 v26, s[42:43], v10, v50\n"\
      "v_cndmask_b32_e64 v42, v24, v40, s[38:39]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v27, s[44:45], v11, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v43, v25, v41, s[38:39]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v26, s[42:43], v26, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[80:81]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v52, s[42:43]\n"\
      "v_lshrrev_b32 v52, 16, v81\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_sub_co_u32_e64 v24, s[36:37], v8, v42\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_subb_co_u32_e64 v25, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_mov_b32 v55, v48\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v24, s[36:37], v24, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[28:29]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[30:31]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[34:35]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[36:37]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[38:39]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v58, v28, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v30, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v32, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v114, v34, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v122, v36, v120, s[74:75]\n"\
      "v_cndmask_b32_e64 v42, v38, v40, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_addc_co_u32_e64 v25, s[24:25], v25, v44, s[36:37]\n"\
      "v_cndmask_b32_e64 v59, v29, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v12, v58\n"\
      "v_cndmask_b32_e64 v99, v31, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v14, v98\n"\
      "v_cndmask_b32_e64 v107, v33, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v16, v106\n"\
      "v_cndmask_b32_e64 v115, v35, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v18, v114\n"\
      "v_cndmask_b32_e64 v123, v37, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v20, v122\n"\
      "v_cndmask_b32_e64 v43, v39, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v22, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_sub_co_u32_e64 v28, s[48:49], v12, v58\n"\
      "v_sub_co_u32_e64 v30, s[54:55], v14, v98\n"\
      "v_sub_co_u32_e64 v32, s[60:61], v16, v106\n"\
      "v_sub_co_u32_e64 v34, s[66:67], v18, v114\n"\
      "v_sub_co_u32_e64 v36, s[72:73], v20, v122\n"\
      "v_sub_co_u32_e64 v38, s[36:37], v22, v42\n"\
      "v_sub_co_u32_e64 v80, s[42:43], v64, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v13, v59, s[52:53]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v15, v99, s[58:59]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v17, v107, s[64:65]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v19, v115, s[70:71]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v21, v123, s[76:77]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v23, v43, s[40:41]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v29, s[50:51], v13, v59, s[48:49]\n"\
      "v_subb_co_u32_e64 v31, s[56:57], v15, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v33, s[62:63], v17, v107, s[60:61]\n"\
      "v_subb_co_u32_e64 v35, s[68:69], v19, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v37, s[74:75], v21, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v39, s[38:39], v23, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v81, s[44:45], v65, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v28, s[48:49], v28, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v30, s[54:55], v30, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v32, s[60:61], v32, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v34, s[66:67], v34, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v36, s[72:73], v36, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v38, s[36:37], v38, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v80, s[42:43], v80, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v109, 1, v[104:105]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v117, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[20:21], s[24:25], v125, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v29, s[24:25], v29, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v31, s[24:25], v31, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v33, s[24:25], v33, v108, s[60:61]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v37, s[24:25], v37, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v39, s[24:25], v39, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v52, s[42:43]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[82:83]\n"\
      "v_lshlrev_b64 v[96:97], 16, v[84:85]\n"\
      "v_lshlrev_b64 v[104:105], 16, v[86:87]\n"\
      "v_lshlrev_b64 v[112:113], 16, v[88:89]\n"\
      "v_lshlrev_b64 v[120:121], 16, v[90:91]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[92:93]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[94:95]\n"\
      "v_lshrrev_b32 v60, 16, v83\n"\
      "v_lshrrev_b32 v100, 16, v85\n"\
      "v_lshrrev_b32 v108, 16, v87\n"\
      "v_lshrrev_b32 v116, 16, v89\n"\
      "v_lshrrev_b32 v124, 16, v91\n"\
      "v_lshrrev_b32 v44, 16, v93\n"\
      "v_lshrrev_b32 v52, 16, v95\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v44, -1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[36:37]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v100, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v108, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v102, 0\n"\
      "v_mov_b32 v103, v96\n"\
      "v_mov_b32 v110, 0\n"\
      "v_mov_b32 v111, v104\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mov_b32 v54, 0\n"\
      "v_mov_b32 v55, v48\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v97, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v105, -1, v[110:111]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v49, -1, v[54:55]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v66, v58\n"\
      "v_sub_co_u32_e64 v82, s[48:49], v66, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v68, v98\n"\
      "v_sub_co_u32_e64 v84, s[54:55], v68, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v70, v106\n"\
      "v_sub_co_u32_e64 v86, s[60:61], v70, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v72, v114\n"\
      "v_sub_co_u32_e64 v88, s[66:67], v72, v114\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v74, v122\n"\
      "v_sub_co_u32_e64 v90, s[72:73], v74, v122\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v76, v42\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v76, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v78, v50\n"\
      "v_sub_co_u32_e64 v94, s[42:43], v78, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v67, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v83, s[50:51], v67, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v69, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v85, s[56:57], v69, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v71, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v87, s[62:63], v71, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v73, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v89, s[68:69], v73, v115, s[66:67]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v75, v123, s[76:77]\n"\
      "v_subb_co_u32_e64 v91, s[74:75], v75, v123, s[72:73]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v77, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v77, v43, s[36:37]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v79, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v95, s[44:45], v79, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v82, s[48:49], v82, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v84, s[54:55], v84, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v86, s[60:61], v86, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v88, s[66:67], v88, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v90, s[72:73], v90, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v94, s[42:43], v94, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[76:77], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[18:19]\n"\
      "v_lshlrev_b64 v[104:105], 16, v[32:33]\n"\
      "v_cndmask_b32_e64 v42, v16, v40, s[38:39]\n"\
      "v_cndmask_b32_e64 v43, v17, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_sub_co_u32_e64 v16, s[36:37], v8, v42\n"\
      "v_cndmask_b32_e64 v50, v18, v48, s[44:45]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v17, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v51, v19, v49, s[44:45]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v16, s[36:37], v16, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_addc_co_u32_e64 v17, s[24:25], v17, v44, s[36:37]\n"\
      "v_sub_co_u32_e64 v18, s[42:43], v10, v50\n"\
      "v_lshlrev_b64 v[112:113], 16, v[34:35]\n"\
      "v_lshlrev_b64 v[120:121], 16, v[36:37]\n"\
      "v_lshlrev_b64 v[40:41], 16, v[38:39]\n"\
      "v_lshrrev_b32 v108, 16, v33\n"\
      "v_lshrrev_b32 v116, 16, v35\n"\
      "v_lshrrev_b32 v124, 16, v37\n"\
      "v_lshrrev_b32 v44, 16, v39\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_subb_co_u32_e64 v19, s[44:45], v11, v51, s[42:43]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v44, -1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v18, s[42:43], v18, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v108, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b64 v[48:49], 24, v[72:73]\n"\
      "v_mov_b32 v110, 0\n"\
      "v_mov_b32 v111, v104\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_lshrrev_b32 v52, 8, v73\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v105, -1, v[110:111]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v41, -1, v[46:47]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[22:23]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v58, v20, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v98, v22, v96, s[56:57]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v26, v114\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v28, v122\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v30, v42\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_sub_co_u32_e64 v34, s[66:67], v26, v114\n"\
      "v_sub_co_u32_e64 v36, s[72:73], v28, v122\n"\
      "v_sub_co_u32_e64 v38, s[36:37], v30, v42\n"\
      "v_sub_co_u32_e64 v72, s[42:43], v64, v50\n"\
      "v_cndmask_b32_e64 v59, v21, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v12, v58\n"\
      "v_cndmask_b32_e64 v99, v23, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v14, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v24, v106\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v27, v115, s[70:71]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v29, v123, s[76:77]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v31, v43, s[40:41]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v20, s[48:49], v12, v58\n"\
      "v_sub_co_u32_e64 v22, s[54:55], v14, v98\n"\
      "v_sub_co_u32_e64 v32, s[60:61], v24, v106\n"\
      "v_subb_co_u32_e64 v35, s[68:69], v27, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v37, s[74:75], v29, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v39, s[38:39], v31, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v73, s[44:45], v65, v51, s[42:43]\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v13, v59, s[52:53]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v15, v99, s[58:59]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v25, v107, s[64:65]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v21, s[50:51], v13, v59, s[48:49]\n"\
      "v_subb_co_u32_e64 v23, s[56:57], v15, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v33, s[62:63], v25, v107, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v34, s[66:67], v34, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v36, s[72:73], v36, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v38, s[36:37], v38, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v72, s[42:43], v72, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v117, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v125, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v20, s[48:49], v20, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v22, s[54:55], v22, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v32, s[60:61], v32, 0, s[62:63]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v37, s[24:25], v37, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v39, s[24:25], v39, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v61, 1, v[56:57]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v109, 1, v[104:105]\n"\
      "v_lshrrev_b64 v[112:113], 24, v[88:89]\n"\
      "v_lshrrev_b64 v[120:121], 24, v[90:91]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[92:93]\n"\
      "v_lshrrev_b64 v[48:49], 24, v[94:95]\n"\
      "v_addc_co_u32_e64 v21, s[24:25], v21, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v23, s[24:25], v23, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v33, s[24:25], v33, v108, s[60:61]\n"\
      "v_lshlrev_b32 v116, 8, v88\n"\
      "v_lshlrev_b32 v124, 8, v90\n"\
      "v_lshlrev_b32 v44, 8, v92\n"\
      "v_lshlrev_b32 v52, 8, v94\n"\
      "v_lshlrev_b64 v[56:57], 24, v[74:75]\n"\
      "v_lshlrev_b64 v[96:97], 24, v[76:77]\n"\
      "v_lshlrev_b64 v[104:105], 24, v[78:79]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v116, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v124, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_lshrrev_b32 v60, 8, v75\n"\
      "v_lshrrev_b32 v100, 8, v77\n"\
      "v_lshrrev_b32 v108, 8, v79\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_sub_co_u32_e64 v115, s[66:67], v115, v116\n"\
      "v_sub_co_u32_e64 v123, s[72:73], v123, v124\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[42:43], v51, v52\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[66:67]\n"\
      "v_addc_co_u32_e64 v114, s[68:69], v114, 0, s[66:67]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v122, s[74:75], v122, 0, s[72:73]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v50, s[44:45], v50, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "v_addc_co_u32_e64 v115, s[24:25], v115, v117, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v80, v114\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v125, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v82, v122\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v84, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v86, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v66, v58\n"\
      "v_sub_co_u32_e64 v74, s[48:49], v66, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v68, v98\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v68, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v70, v106\n"\
      "v_sub_co_u32_e64 v78, s[60:61], v70, v106\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v81, v115, s[70:71]\n"\
      "v_sub_co_u32_e64 v80, s[66:67], v80, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v83, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v82, s[72:73], v82, v122\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v85, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v84, s[36:37], v84, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v87, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v86, s[42:43], v86, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v67, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v75, s[50:51], v67, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v69, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v69, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v71, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v79, s[62:63], v71, v107, s[60:61]\n"\
      "v_subb_co_u32_e64 v81, s[68:69], v81, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v83, s[74:75], v83, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v85, s[38:39], v85, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v87, s[44:45], v87, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v74, s[48:49], v74, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v78, s[60:61], v78, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v80, s[66:67], v80, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v82, s[72:73], v82, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v84, s[36:37], v84, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v86, s[42:43], v86, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[70:71], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[90:91], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v53, 1, v[48:49]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[12:13]\n"\
      "v_lshlrev_b64 v[56:57], 16, v[20:21]\n"\
      "v_lshlrev_b64 v[96:97], 16, v[22:23]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[14:15]\n"\
      "v_lshrrev_b32 v60, 16, v21\n"\
      "v_lshrrev_b32 v100, 16, v23\n"\
      "v_cndmask_b32_e64 v42, v12, v40, s[38:39]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_cndmask_b32_e64 v50, v14, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v43, v13, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_sub_co_u32_e64 v12, s[36:37], v8, v42\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v51, v15, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v10, v50\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v14, s[42:43], v10, v50\n"\
      "v_subb_co_u32_e64 v13, s[38:39], v9, v43, s[36:37]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v100, 1, v[98:99]\n"\
      "v_lshrrev_b64 v[120:121], 24, v[36:37]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v11, v51, s[46:47]\n"\
      "v_lshlrev_b32 v124, 8, v36\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v15, s[44:45], v11, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[104:105], 24, v[28:29]\n"\
      "v_lshlrev_b64 v[112:113], 24, v[30:31]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v12, s[36:37], v12, 0, s[38:39]\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_mov_b32 v102, 0\n"\
      "v_mov_b32 v103, v96\n"\
      "v_lshrrev_b32 v108, 8, v29\n"\
      "v_lshrrev_b32 v116, 8, v31\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v124, 1, v[120:121]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v14, s[42:43], v14, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v97, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_addc_co_u32_e64 v13, s[24:25], v13, v44, s[36:37]\n"\
      "v_sub_co_u32_e64 v123, s[72:73], v123, v124\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v15, s[24:25], v15, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_lshrrev_b64 v[40:41], 24, v[38:39]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v122, s[74:75], v122, 0, s[72:73]\n"\
      "v_lshlrev_b32 v44, 8, v38\n"\
      "v_lshlrev_b64 v[48:49], 12, v[68:69]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_lshrrev_b32 v52, 20, v69\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v125, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v32, v122\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v18, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v24, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v26, v114\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_sub_co_u32_e64 v22, s[54:55], v18, v98\n"\
      "v_sub_co_u32_e64 v28, s[60:61], v24, v106\n"\
      "v_sub_co_u32_e64 v30, s[66:67], v26, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v33, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v32, s[72:73], v32, v122\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v19, v99, s[58:59]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v25, v107, s[64:65]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v27, v115, s[70:71]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v23, s[56:57], v19, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v29, s[62:63], v25, v107, s[60:61]\n"\
      "v_subb_co_u32_e64 v31, s[68:69], v27, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v33, s[74:75], v33, v123, s[72:73]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v34, v42\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v22, s[54:55], v22, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v28, s[60:61], v28, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v30, s[66:67], v30, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v32, s[72:73], v32, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v109, 1, v[104:105]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v117, 1, v[112:113]\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v35, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v34, s[36:37], v34, v42\n"\
      "v_sub_co_u32_e64 v68, s[42:43], v64, v50\n"\
      "v_addc_co_u32_e64 v23, s[24:25], v23, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v29, s[24:25], v29, v108, s[60:61]\n"\
      "v_addc_co_u32_e64 v31, s[24:25], v31, v116, s[66:67]\n"\
      "v_addc_co_u32_e64 v33, s[24:25], v33, v124, s[72:73]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v16, v58\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v20, s[48:49], v16, v58\n"\
      "v_subb_co_u32_e64 v35, s[38:39], v35, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v69, s[44:45], v65, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[96:97], 28, v[76:77]\n"\
      "v_lshlrev_b64 v[104:105], 28, v[78:79]\n"\
      "v_lshlrev_b64 v[112:113], 4, v[84:85]\n"\
      "v_lshlrev_b64 v[120:121], 4, v[86:87]\n"\
      "v_lshrrev_b32 v100, 4, v77\n"\
      "v_lshrrev_b32 v108, 4, v79\n"\
      "v_lshrrev_b32 v116, 28, v85\n"\
      "v_lshrrev_b32 v124, 28, v87\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v17, v59, s[52:53]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v21, s[50:51], v17, v59, s[48:49]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v34, s[36:37], v34, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v68, s[42:43], v68, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v45, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v20, s[48:49], v20, 0, s[50:51]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[54:55]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v61, 1, v[56:57]\n"\
      "v_lshrrev_b64 v[40:41], 12, v[92:93]\n"\
      "v_lshrrev_b64 v[48:49], 12, v[94:95]\n"\
      "v_addc_co_u32_e64 v21, s[24:25], v21, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v100, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[24:25], v108, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_lshlrev_b32 v44, 20, v92\n"\
      "v_lshlrev_b32 v52, 20, v94\n"\
      "v_lshlrev_b64 v[56:57], 12, v[70:71]\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_lshrrev_b32 v60, 20, v71\n"\
      "v_mov_b32 v102, 0\n"\
      "v_mov_b32 v103, v96\n"\
      "v_mov_b32 v110, 0\n"\
      "v_mov_b32 v111, v104\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v97, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v105, -1, v[110:111]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_sub_co_u32_e64 v51, s[42:43], v51, v52\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v50, s[44:45], v50, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v88, v42\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v90, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v66, v58\n"\
      "v_sub_co_u32_e64 v70, s[48:49], v66, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v72, v98\n"\
      "v_sub_co_u32_e64 v76, s[54:55], v72, v98\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v74, v106\n"\
      "v_sub_co_u32_e64 v78, s[60:61], v74, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v80, v114\n"\
      "v_sub_co_u32_e64 v84, s[66:67], v80, v114\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v82, v122\n"\
      "v_sub_co_u32_e64 v86, s[72:73], v82, v122\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v89, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v88, s[36:37], v88, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v91, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v90, s[42:43], v90, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v67, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v71, s[50:51], v67, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v73, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v77, s[56:57], v73, v99, s[54:55]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v75, v107, s[64:65]\n"\
      "v_subb_co_u32_e64 v79, s[62:63], v75, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v81, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v85, s[68:69], v81, v115, s[66:67]\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v83, v123, s[76:77]\n"\
      "v_subb_co_u32_e64 v87, s[74:75], v83, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v89, s[38:39], v89, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v91, s[44:45], v91, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v70, s[48:49], v70, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v76, s[54:55], v76, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v78, s[60:61], v78, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v84, s[66:67], v84, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v86, s[72:73], v86, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v88, s[36:37], v88, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v90, s[42:43], v90, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[66:67], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[74:75], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[82:83], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[92:93], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v53, 1, v[48:49]\n"\
      "v_lshlrev_b64 v[48:49], 16, v[14:15]\n"\
      "v_lshrrev_b32 v52, 16, v15\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[10:11]\n"\
      "v_mov_b32 v54, 0\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[42:43]\n"\
      "v_mad_u64_u32 v[48:49], s[24:25], v52, 1, v[50:51]\n"\
      "v_cndmask_b32_e64 v42, v10, v40, s[38:39]\n"\
      "v_mov_b32 v55, v48\n"\
      "v_cndmask_b32_e64 v43, v11, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v8, v42\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v49, -1, v[54:55]\n"\
      "v_sub_co_u32_e64 v10, s[36:37], v8, v42\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v9, v43, s[40:41]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_subb_co_u32_e64 v11, s[38:39], v9, v43, s[36:37]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v10, s[36:37], v10, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v45, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v12, v50\n"\
      "v_addc_co_u32_e64 v11, s[24:25], v11, v44, s[36:37]\n"\
      "v_sub_co_u32_e64 v14, s[42:43], v12, v50\n"\
      "v_lshlrev_b64 v[112:113], 28, v[30:31]\n"\
      "v_lshlrev_b64 v[120:121], 4, v[34:35]\n"\
      "v_lshrrev_b32 v116, 4, v31\n"\
      "v_lshrrev_b32 v124, 28, v35\n"\
      "v_lshrrev_b64 v[40:41], 12, v[38:39]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v13, v51, s[46:47]\n"\
      "v_lshlrev_b32 v44, 20, v38\n"\
      "v_subb_co_u32_e64 v15, s[44:45], v13, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[56:57], 24, v[18:19]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v124, -1, v[120:121]\n"\
      "v_lshrrev_b32 v60, 8, v19\n"\
      "v_mad_u64_u32 v[42:43], s[24:25], v44, 1, v[40:41]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v14, s[42:43], v14, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[72:73]\n"\
      "v_sub_co_u32_e64 v43, s[36:37], v43, v44\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v53, 1, v[48:49]\n"\
      "v_addc_co_u32_e64 v15, s[24:25], v15, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v116, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[24:25], v124, 1, v[122:123]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[36:37]\n"\
      "v_addc_co_u32_e64 v42, s[38:39], v42, 0, s[36:37]\n"\
      "v_lshlrev_b64 v[104:105], 12, v[26:27]\n"\
      "v_lshlrev_b64 v[48:49], 6, v[66:67]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "v_lshrrev_b64 v[96:97], 24, v[22:23]\n"\
      "v_lshrrev_b32 v108, 20, v27\n"\
      "v_mov_b32 v118, 0\n"\
      "v_mov_b32 v119, v112\n"\
      "v_mov_b32 v126, 0\n"\
      "v_mov_b32 v127, v120\n"\
      "v_lshrrev_b32 v52, 26, v67\n"\
      "v_lshlrev_b32 v100, 8, v22\n"\
      "v_addc_co_u32_e64 v43, s[24:25], v43, v45, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v36, v42\n"\
      "v_mad_u64_u32 v[106:107], s[60:61], v108, -1, v[104:105]\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v113, -1, v[118:119]\n"\
      "v_mad_u64_u32 v[122:123], s[72:73], v121, -1, v[126:127]\n"\
      "v_mad_u64_u32 v[50:51], s[42:43], v52, -1, v[48:49]\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v16, v58\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v100, 1, v[96:97]\n"\
      "v_sub_co_u32_e64 v18, s[48:49], v16, v58\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v37, v43, s[40:41]\n"\
      "v_sub_co_u32_e64 v36, s[36:37], v36, v42\n"\
      "v_mad_u64_u32 v[104:105], s[62:63], -1, 1, v[106:107]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_mad_u64_u32 v[120:121], s[74:75], -1, 1, v[122:123]\n"\
      "v_mad_u64_u32 v[48:49], s[44:45], -1, 1, v[50:51]\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v17, v59, s[52:53]\n"\
      "v_sub_co_u32_e64 v99, s[54:55], v99, v100\n"\
      "v_subb_co_u32_e64 v19, s[50:51], v17, v59, s[48:49]\n"\
      "v_subb_co_u32_e64 v37, s[38:39], v37, v43, s[36:37]\n"\
      "s_or_b64 s[62:63], s[62:63], s[60:61]\n"\
      "v_cndmask_b32_e64 v106, v106, v104, s[62:63]\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "s_or_b64 s[74:75], s[74:75], s[72:73]\n"\
      "v_cndmask_b32_e64 v122, v122, v120, s[74:75]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v50, v50, v48, s[44:45]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[54:55]\n"\
      "v_addc_co_u32_e64 v98, s[56:57], v98, 0, s[54:55]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v18, s[48:49], v18, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v36, s[36:37], v36, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v107, v107, v105, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v24, v106\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "v_cndmask_b32_e64 v123, v123, v121, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v32, v122\n"\
      "v_cndmask_b32_e64 v51, v51, v49, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v64, v50\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v99, s[24:25], v99, v101, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v20, v98\n"\
      "v_sub_co_u32_e64 v26, s[60:61], v24, v106\n"\
      "v_sub_co_u32_e64 v34, s[72:73], v32, v122\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v45, 1, v[40:41]\n"\
      "v_sub_co_u32_e64 v66, s[42:43], v64, v50\n"\
      "v_addc_co_u32_e64 v19, s[24:25], v19, v60, s[48:49]\n"\
      "v_addc_co_u32_e64 v37, s[24:25], v37, v44, s[36:37]\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v25, v107, s[64:65]\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v28, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v33, v123, s[76:77]\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v65, v51, s[46:47]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v21, v99, s[58:59]\n"\
      "v_sub_co_u32_e64 v20, s[54:55], v20, v98\n"\
      "v_subb_co_u32_e64 v27, s[62:63], v25, v107, s[60:61]\n"\
      "v_sub_co_u32_e64 v30, s[66:67], v28, v114\n"\
      "v_subb_co_u32_e64 v35, s[74:75], v33, v123, s[72:73]\n"\
      "v_subb_co_u32_e64 v67, s[44:45], v65, v51, s[42:43]\n"\
      "v_lshlrev_b64 v[56:57], 22, v[70:71]\n"\
      "v_lshlrev_b64 v[40:41], 10, v[90:91]\n"\
      "v_lshrrev_b32 v60, 10, v71\n"\
      "v_lshrrev_b32 v44, 22, v91\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v29, v115, s[70:71]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_subb_co_u32_e64 v21, s[56:57], v21, v99, s[54:55]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v26, s[60:61], v26, 0, s[62:63]\n"\
      "v_subb_co_u32_e64 v31, s[68:69], v29, v115, s[66:67]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v34, s[72:73], v34, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v66, s[42:43], v66, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v60, -1, v[56:57]\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v44, -1, v[40:41]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v109, 1, v[104:105]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v125, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[64:65], s[24:25], v53, 1, v[48:49]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v20, s[54:55], v20, 0, s[56:57]\n"\
      "v_addc_co_u32_e64 v27, s[24:25], v27, v108, s[60:61]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v30, s[66:67], v30, 0, s[68:69]\n"\
      "v_addc_co_u32_e64 v35, s[24:25], v35, v124, s[72:73]\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v52, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[48:49]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[36:37]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v101, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v117, 1, v[112:113]\n"\
      "v_lshrrev_b64 v[104:105], 18, v[78:79]\n"\
      "v_lshrrev_b64 v[120:121], 30, v[86:87]\n"\
      "v_lshrrev_b64 v[48:49], 6, v[94:95]\n"\
      "v_addc_co_u32_e64 v21, s[24:25], v21, v100, s[54:55]\n"\
      "v_addc_co_u32_e64 v31, s[24:25], v31, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[56:57], s[24:25], v60, 1, v[58:59]\n"\
      "v_lshlrev_b32 v108, 14, v78\n"\
      "v_lshlrev_b32 v124, 2, v86\n"\
      "v_mad_u64_u32 v[40:41], s[24:25], v44, 1, v[42:43]\n"\
      "v_lshlrev_b32 v52, 26, v94\n"\
      "v_lshlrev_b64 v[96:97], 30, v[74:75]\n"\
      "v_mad_u64_u32 v[106:107], s[24:25], v108, 1, v[104:105]\n"\
      "v_lshlrev_b64 v[112:113], 18, v[82:83]\n"\
      "v_mad_u64_u32 v[122:123], s[24:25], v124, 1, v[120:121]\n"\
      "v_mad_u64_u32 v[50:51], s[24:25], v52, 1, v[48:49]\n"\
      "v_mov_b32 v62, 0\n"\
      "v_mov_b32 v63, v56\n"\
      "v_lshrrev_b32 v100, 2, v75\n"\
      "v_lshrrev_b32 v116, 14, v83\n"\
      "v_mov_b32 v46, 0\n"\
      "v_mov_b32 v47, v40\n"\
      "v_mad_u64_u32 v[58:59], s[48:49], v57, -1, v[62:63]\n"\
      "v_mad_u64_u32 v[98:99], s[54:55], v100, -1, v[96:97]\n"\
      "v_sub_co_u32_e64 v107, s[60:61], v107, v108\n"\
      "v_mad_u64_u32 v[114:115], s[66:67], v116, -1, v[112:113]\n"\
      "v_sub_co_u32_e64 v123, s[72:73], v123, v124\n"\
      "v_mad_u64_u32 v[42:43], s[36:37], v41, -1, v[46:47]\n"\
      "v_sub_co_u32_e64 v51, s[42:43], v51, v52\n"\
      "v_mad_u64_u32 v[56:57], s[50:51], -1, 1, v[58:59]\n"\
      "v_mad_u64_u32 v[96:97], s[56:57], -1, 1, v[98:99]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[60:61]\n"\
      "v_addc_co_u32_e64 v106, s[62:63], v106, 0, s[60:61]\n"\
      "v_mad_u64_u32 v[112:113], s[68:69], -1, 1, v[114:115]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[72:73]\n"\
      "v_addc_co_u32_e64 v122, s[74:75], v122, 0, s[72:73]\n"\
      "v_mad_u64_u32 v[40:41], s[38:39], -1, 1, v[42:43]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[42:43]\n"\
      "v_addc_co_u32_e64 v50, s[44:45], v50, 0, s[42:43]\n"\
      "s_or_b64 s[50:51], s[50:51], s[48:49]\n"\
      "v_cndmask_b32_e64 v58, v58, v56, s[50:51]\n"\
      "s_or_b64 s[56:57], s[56:57], s[54:55]\n"\
      "v_cndmask_b32_e64 v98, v98, v96, s[56:57]\n"\
      "v_addc_co_u32_e64 v107, s[24:25], v107, v109, s[62:63]\n"\
      "v_add_co_u32_e64 v104, s[64:65], v76, v106\n"\
      "s_or_b64 s[68:69], s[68:69], s[66:67]\n"\
      "v_cndmask_b32_e64 v114, v114, v112, s[68:69]\n"\
      "v_addc_co_u32_e64 v123, s[24:25], v123, v125, s[74:75]\n"\
      "v_add_co_u32_e64 v120, s[76:77], v84, v122\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v42, v42, v40, s[38:39]\n"\
      "v_addc_co_u32_e64 v51, s[24:25], v51, v53, s[44:45]\n"\
      "v_add_co_u32_e64 v48, s[46:47], v92, v50\n"\
      "v_cndmask_b32_e64 v59, v59, v57, s[50:51]\n"\
      "v_add_co_u32_e64 v56, s[52:53], v68, v58\n"\
      "v_sub_co_u32_e64 v70, s[48:49], v68, v58\n"\
      "v_cndmask_b32_e64 v99, v99, v97, s[56:57]\n"\
      "v_add_co_u32_e64 v96, s[58:59], v72, v98\n"\
      "v_sub_co_u32_e64 v74, s[54:55], v72, v98\n"\
      "v_addc_co_u32_e64 v105, s[64:65], v77, v107, s[64:65]\n"\
      "v_sub_co_u32_e64 v76, s[60:61], v76, v106\n"\
      "v_cndmask_b32_e64 v115, v115, v113, s[68:69]\n"\
      "v_add_co_u32_e64 v112, s[70:71], v80, v114\n"\
      "v_sub_co_u32_e64 v82, s[66:67], v80, v114\n"\
      "v_addc_co_u32_e64 v121, s[76:77], v85, v123, s[76:77]\n"\
      "v_sub_co_u32_e64 v84, s[72:73], v84, v122\n"\
      "v_cndmask_b32_e64 v43, v43, v41, s[38:39]\n"\
      "v_add_co_u32_e64 v40, s[40:41], v88, v42\n"\
      "v_sub_co_u32_e64 v90, s[36:37], v88, v42\n"\
      "v_addc_co_u32_e64 v49, s[46:47], v93, v51, s[46:47]\n"\
      "v_sub_co_u32_e64 v92, s[42:43], v92, v50\n"\
      "v_addc_co_u32_e64 v57, s[52:53], v69, v59, s[52:53]\n"\
      "v_subb_co_u32_e64 v71, s[50:51], v69, v59, s[48:49]\n"\
      "v_addc_co_u32_e64 v97, s[58:59], v73, v99, s[58:59]\n"\
      "v_subb_co_u32_e64 v75, s[56:57], v73, v99, s[54:55]\n"\
      "v_subb_co_u32_e64 v77, s[62:63], v77, v107, s[60:61]\n"\
      "v_addc_co_u32_e64 v113, s[70:71], v81, v115, s[70:71]\n"\
      "v_subb_co_u32_e64 v83, s[68:69], v81, v115, s[66:67]\n"\
      "v_subb_co_u32_e64 v85, s[74:75], v85, v123, s[72:73]\n"\
      "v_addc_co_u32_e64 v41, s[40:41], v89, v43, s[40:41]\n"\
      "v_subb_co_u32_e64 v91, s[38:39], v89, v43, s[36:37]\n"\
      "v_subb_co_u32_e64 v93, s[44:45], v93, v51, s[42:43]\n"\
      "v_cndmask_b32_e64 v60, 0, -1, s[50:51]\n"\
      "v_addc_co_u32_e64 v70, s[48:49], v70, 0, s[50:51]\n"\
      "v_cndmask_b32_e64 v61, 0, -1, s[52:53]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[56:57]\n"\
      "v_addc_co_u32_e64 v74, s[54:55], v74, 0, s[56:57]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[58:59]\n"\
      "v_cndmask_b32_e64 v108, 0, -1, s[62:63]\n"\
      "v_addc_co_u32_e64 v76, s[60:61], v76, 0, s[62:63]\n"\
      "v_cndmask_b32_e64 v109, 0, -1, s[64:65]\n"\
      "v_cndmask_b32_e64 v116, 0, -1, s[68:69]\n"\
      "v_addc_co_u32_e64 v82, s[66:67], v82, 0, s[68:69]\n"\
      "v_cndmask_b32_e64 v117, 0, -1, s[70:71]\n"\
      "v_cndmask_b32_e64 v124, 0, -1, s[74:75]\n"\
      "v_addc_co_u32_e64 v84, s[72:73], v84, 0, s[74:75]\n"\
      "v_cndmask_b32_e64 v125, 0, -1, s[76:77]\n"\
      "v_cndmask_b32_e64 v44, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v90, s[36:37], v90, 0, s[38:39]\n"\
      "v_cndmask_b32_e64 v45, 0, -1, s[40:41]\n"\
      "v_cndmask_b32_e64 v52, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v92, s[42:43], v92, 0, s[44:45]\n"\
      "v_cndmask_b32_e64 v53, 0, -1, s[46:47]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v60, s[48:49]\n"\
      "v_mad_u64_u32 v[68:69], s[24:25], v61, 1, v[56:57]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v100, s[54:55]\n"\
      "v_mad_u64_u32 v[72:73], s[24:25], v101, 1, v[96:97]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v108, s[60:61]\n"\
      "v_mad_u64_u32 v[78:79], s[24:25], v109, 1, v[104:105]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v116, s[66:67]\n"\
      "v_mad_u64_u32 v[80:81], s[24:25], v117, 1, v[112:113]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v124, s[72:73]\n"\
      "v_mad_u64_u32 v[86:87], s[24:25], v125, 1, v[120:121]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v44, s[36:37]\n"\
      "v_mad_u64_u32 v[88:89], s[24:25], v45, 1, v[40:41]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v52, s[42:43]\n"\
      "v_mad_u64_u32 v[94:95], s[24:25], v53, 1, v[48:49]\n"\
      "global_load_dwordx2 v[40:41], %[lwo], %[lw] offset:0\n"\
      "global_load_dwordx2 v[42:43], %[lwo], %[lw] offset:8\n"\
      "global_load_dwordx2 v[44:45], %[lwo], %[lw] offset:16\n"\
      "global_load_dwordx2 v[46:47], %[lwo], %[lw] offset:24\n"\
      "global_load_dwordx2 v[48:49], %[lwo], %[lw] offset:32\n"\
      "global_load_dwordx2 v[50:51], %[lwo], %[lw] offset:40\n"\
      "global_load_dwordx2 v[52:53], %[lwo], %[lw] offset:48\n"\
      "global_load_dwordx2 v[54:55], %[lwo], %[lw] offset:56\n"\
      "s_waitcnt vmcnt(0)\n"\
      "s_nop 1\n"\
      "v_mov_b32_dpp v56, v8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v64 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v66 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v64, v56, v64, s[20:21]\n"\
      "v_cndmask_b32_e64 v66, v60, v66, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v64, v40, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v66, v42, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v65 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v64, v41, v[104:105]\n"\
      "v_mov_b32_dpp v61, v11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v67 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v66, v43, v[116:117]\n"\
      "v_cndmask_b32_e64 v65, v57, v65, s[20:21]\n"\
      "v_cndmask_b32_e64 v67, v61, v67, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v65, v40, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v65, v41, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v67, v42, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v67, v43, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v8, v8, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v10, v10, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v9, v9, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v8, v104\n"\
      "v_cndmask_b32_e64 v11, v11, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v10, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v9, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v64, s[36:37], v8, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v11, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v66, s[42:43], v10, v116\n"\
      "v_subb_co_u32_e64 v65, s[38:39], v9, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v67, s[44:45], v11, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v64, s[36:37], v64, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[8:9], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v66, s[42:43], v66, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[10:11], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[8:9]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[10:11]\n"\
      "v_addc_co_u32_e64 v65, s[24:25], v65, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v8, v8, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v9, v9, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v67, s[24:25], v67, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v10, v10, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v11, v11, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[64:65]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[66:67]\n"\
      "v_mov_b32_dpp v56, v12 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v68 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v14 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v70 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v64, v64, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v65, v65, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v66, v66, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v67, v67, v109, s[44:45]\n"\
      "v_cndmask_b32_e64 v68, v56, v68, s[20:21]\n"\
      "v_cndmask_b32_e64 v70, v60, v70, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v68, v44, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v70, v46, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v13 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v69 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v68, v45, v[104:105]\n"\
      "v_mov_b32_dpp v61, v15 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v71 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v70, v47, v[116:117]\n"\
      "v_cndmask_b32_e64 v69, v57, v69, s[20:21]\n"\
      "v_cndmask_b32_e64 v71, v61, v71, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v69, v44, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v69, v45, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v71, v46, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v71, v47, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v12, v12, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v14, v14, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v13, v13, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v12, v104\n"\
      "v_cndmask_b32_e64 v15, v15, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v14, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v13, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v68, s[36:37], v12, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v15, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v70, s[42:43], v14, v116\n"\
      "v_subb_co_u32_e64 v69, s[38:39], v13, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v71, s[44:45], v15, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v68, s[36:37], v68, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[12:13], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v70, s[42:43], v70, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[14:15], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[12:13]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[14:15]\n"\
      "v_addc_co_u32_e64 v69, s[24:25], v69, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v12, v12, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v13, v13, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v71, s[24:25], v71, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v14, v14, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v15, v15, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[68:69]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[70:71]\n"\
      "v_mov_b32_dpp v56, v16 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v72 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v18 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v74 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v68, v68, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v69, v69, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v70, v70, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v71, v71, v109, s[44:45]\n"\
      "v_cndmask_b32_e64 v72, v56, v72, s[20:21]\n"\
      "v_cndmask_b32_e64 v74, v60, v74, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v72, v48, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v74, v50, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v73 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v72, v49, v[104:105]\n"\
      "v_mov_b32_dpp v61, v19 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v75 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v74, v51, v[116:117]\n"\
      "v_cndmask_b32_e64 v73, v57, v73, s[20:21]\n"\
      "v_cndmask_b32_e64 v75, v61, v75, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v73, v48, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v73, v49, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v75, v50, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v75, v51, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v16, v16, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v17, v17, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v16, v104\n"\
      "v_cndmask_b32_e64 v19, v19, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v18, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v17, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v72, s[36:37], v16, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v19, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v74, s[42:43], v18, v116\n"\
      "v_subb_co_u32_e64 v73, s[38:39], v17, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v75, s[44:45], v19, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v72, s[36:37], v72, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[16:17], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v74, s[42:43], v74, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[18:19], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[16:17]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[18:19]\n"\
      "v_addc_co_u32_e64 v73, s[24:25], v73, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v16, v16, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v17, v17, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v75, s[24:25], v75, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v18, v18, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v19, v19, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[72:73]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[74:75]\n"\
      "v_mov_b32_dpp v56, v20 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v76 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v22 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v78 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v72, v72, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v73, v73, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v74, v74, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v75, v75, v109, s[44:45]\n"\
      "v_cndmask_b32_e64 v76, v56, v76, s[20:21]\n"\
      "v_cndmask_b32_e64 v78, v60, v78, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v76, v52, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v78, v54, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v21 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v77 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v76, v53, v[104:105]\n"\
      "v_mov_b32_dpp v61, v23 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v79 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v78, v55, v[116:117]\n"\
      "v_cndmask_b32_e64 v77, v57, v77, s[20:21]\n"\
      "v_cndmask_b32_e64 v79, v61, v79, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v77, v52, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v77, v53, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v79, v54, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v79, v55, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v20, v20, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v22, v22, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v21, v21, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v20, v104\n"\
      "v_cndmask_b32_e64 v23, v23, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v22, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v21, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v76, s[36:37], v20, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v23, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v78, s[42:43], v22, v116\n"\
      "v_subb_co_u32_e64 v77, s[38:39], v21, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v79, s[44:45], v23, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v76, s[36:37], v76, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[20:21], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v78, s[42:43], v78, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[22:23], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[20:21]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[22:23]\n"\
      "v_addc_co_u32_e64 v77, s[24:25], v77, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v20, v20, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v21, v21, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v79, s[24:25], v79, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v22, v22, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v23, v23, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[76:77]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[78:79]\n"\
      "s_nop 0\n"\
      "v_cndmask_b32_e64 v76, v76, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v77, v77, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v78, v78, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v79, v79, v109, s[44:45]\n"\
      "global_load_dwordx2 v[40:41], %[lwo], %[lw] offset:64\n"\
      "global_load_dwordx2 v[42:43], %[lwo], %[lw] offset:72\n"\
      "global_load_dwordx2 v[44:45], %[lwo], %[lw] offset:80\n"\
      "global_load_dwordx2 v[46:47], %[lwo], %[lw] offset:88\n"\
      "global_load_dwordx2 v[48:49], %[lwo], %[lw] offset:96\n"\
      "global_load_dwordx2 v[50:51], %[lwo], %[lw] offset:104\n"\
      "global_load_dwordx2 v[52:53], %[lwo], %[lw] offset:112\n"\
      "global_load_dwordx2 v[54:55], %[lwo], %[lw] offset:120\n"\
      "s_waitcnt vmcnt(0)\n"\
      "s_nop 1\n"\
      "v_mov_b32_dpp v56, v24 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v80 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v26 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v82 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v80, v56, v80, s[20:21]\n"\
      "v_cndmask_b32_e64 v82, v60, v82, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v80, v40, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v82, v42, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v25 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v81 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v80, v41, v[104:105]\n"\
      "v_mov_b32_dpp v61, v27 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v83 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v82, v43, v[116:117]\n"\
      "v_cndmask_b32_e64 v81, v57, v81, s[20:21]\n"\
      "v_cndmask_b32_e64 v83, v61, v83, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v81, v40, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v81, v41, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v83, v42, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v83, v43, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v24, v24, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v26, v26, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v25, v25, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v24, v104\n"\
      "v_cndmask_b32_e64 v27, v27, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v26, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v25, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v80, s[36:37], v24, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v27, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v82, s[42:43], v26, v116\n"\
      "v_subb_co_u32_e64 v81, s[38:39], v25, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v83, s[44:45], v27, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v80, s[36:37], v80, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[24:25], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v82, s[42:43], v82, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[26:27], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[24:25]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[26:27]\n"\
      "v_addc_co_u32_e64 v81, s[24:25], v81, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v24, v24, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v25, v25, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v83, s[24:25], v83, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v26, v26, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v27, v27, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[80:81]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[82:83]\n"\
      "v_mov_b32_dpp v56, v28 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v84 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v30 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v86 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v80, v80, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v81, v81, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v82, v82, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v83, v83, v109, s[44:45]\n"\
      "v_cndmask_b32_e64 v84, v56, v84, s[20:21]\n"\
      "v_cndmask_b32_e64 v86, v60, v86, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v84, v44, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v86, v46, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v29 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v85 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v84, v45, v[104:105]\n"\
      "v_mov_b32_dpp v61, v31 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v87 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v86, v47, v[116:117]\n"\
      "v_cndmask_b32_e64 v85, v57, v85, s[20:21]\n"\
      "v_cndmask_b32_e64 v87, v61, v87, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v85, v44, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v85, v45, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v87, v46, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v87, v47, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v28, v28, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v30, v30, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v29, v29, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v28, v104\n"\
      "v_cndmask_b32_e64 v31, v31, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v30, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v29, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v84, s[36:37], v28, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v31, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v86, s[42:43], v30, v116\n"\
      "v_subb_co_u32_e64 v85, s[38:39], v29, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v87, s[44:45], v31, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v84, s[36:37], v84, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[28:29], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v86, s[42:43], v86, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[30:31], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[28:29]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[30:31]\n"\
      "v_addc_co_u32_e64 v85, s[24:25], v85, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v28, v28, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v29, v29, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v87, s[24:25], v87, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v30, v30, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v31, v31, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[84:85]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[86:87]\n"\
      "v_mov_b32_dpp v56, v32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v88 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v90 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v84, v84, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v85, v85, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v86, v86, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v87, v87, v109, s[44:45]\n"\
      "v_cndmask_b32_e64 v88, v56, v88, s[20:21]\n"\
      "v_cndmask_b32_e64 v90, v60, v90, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v88, v48, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v90, v50, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v33 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v89 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v88, v49, v[104:105]\n"\
      "v_mov_b32_dpp v61, v35 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v91 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v90, v51, v[116:117]\n"\
      "v_cndmask_b32_e64 v89, v57, v89, s[20:21]\n"\
      "v_cndmask_b32_e64 v91, v61, v91, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v89, v48, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v89, v49, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v91, v50, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v91, v51, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v32, v32, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v34, v34, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v33, v33, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v32, v104\n"\
      "v_cndmask_b32_e64 v35, v35, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v34, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v33, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v88, s[36:37], v32, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v35, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v90, s[42:43], v34, v116\n"\
      "v_subb_co_u32_e64 v89, s[38:39], v33, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v91, s[44:45], v35, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v88, s[36:37], v88, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[32:33], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v90, s[42:43], v90, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[34:35], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[32:33]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[34:35]\n"\
      "v_addc_co_u32_e64 v89, s[24:25], v89, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v32, v32, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v33, v33, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v91, s[24:25], v91, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v34, v34, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v35, v35, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[88:89]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[90:91]\n"\
      "v_mov_b32_dpp v56, v36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v58, v92 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v60, v38 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v62, v94 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_cndmask_b32_e64 v88, v88, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v89, v89, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v90, v90, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v91, v91, v109, s[44:45]\n"\
      "v_cndmask_b32_e64 v92, v56, v92, s[20:21]\n"\
      "v_cndmask_b32_e64 v94, v60, v94, s[20:21]\n"\
      "v_mad_u64_u32 v[96:97], s[24:25], v92, v52, 0\n"\
      "v_mad_u64_u32 v[108:109], s[24:25], v94, v54, 0\n"\
      "v_mov_b32 v105, 0\n"\
      "v_mov_b32 v104, v97\n"\
      "v_mov_b32 v117, 0\n"\
      "v_mov_b32 v116, v109\n"\
      "v_mov_b32_dpp v57, v37 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v59, v93 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v92, v53, v[104:105]\n"\
      "v_mov_b32_dpp v61, v39 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mov_b32_dpp v63, v95 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v94, v55, v[116:117]\n"\
      "v_cndmask_b32_e64 v93, v57, v93, s[20:21]\n"\
      "v_cndmask_b32_e64 v95, v61, v95, s[20:21]\n"\
      "v_mov_b32 v107, 0\n"\
      "v_mov_b32 v106, v98\n"\
      "v_mov_b32 v104, v99\n"\
      "v_mov_b32 v119, 0\n"\
      "v_mov_b32 v118, v110\n"\
      "v_mov_b32 v116, v111\n"\
      "v_mad_u64_u32 v[100:101], s[24:25], v93, v52, v[106:107]\n"\
      "v_mad_u64_u32 v[102:103], s[24:25], v93, v53, v[104:105]\n"\
      "v_mad_u64_u32 v[112:113], s[24:25], v95, v54, v[118:119]\n"\
      "v_mad_u64_u32 v[114:115], s[24:25], v95, v55, v[116:117]\n"\
      "v_mad_u64_u32 v[98:99], s[24:25], v101, 1, v[102:103]\n"\
      "v_mad_u64_u32 v[110:111], s[24:25], v113, 1, v[114:115]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v96, v99\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v108, v111\n"\
      "v_cndmask_b32_e64 v36, v36, v58, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[38:39], v100, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[44:45], v112, 0, s[42:43]\n"\
      "v_cndmask_b32_e64 v38, v38, v62, s[20:21]\n"\
      "v_cndmask_b32_e64 v106, 0, -1, s[38:39]\n"\
      "v_cndmask_b32_e64 v118, 0, -1, s[44:45]\n"\
      "v_sub_co_u32_e64 v102, s[36:37], v102, v106\n"\
      "v_sub_co_u32_e64 v114, s[42:43], v114, v118\n"\
      "v_cndmask_b32_e64 v37, v37, v59, s[20:21]\n"\
      "v_subb_co_u32_e64 v103, s[24:25], v103, 0, s[36:37]\n"\
      "v_subb_co_u32_e64 v115, s[24:25], v115, 0, s[42:43]\n"\
      "v_mad_u64_u32 v[96:97], s[36:37], v98, -1, v[102:103]\n"\
      "v_mad_u64_u32 v[108:109], s[42:43], v110, -1, v[114:115]\n"\
      "v_mad_u64_u32 v[100:101], s[38:39], -1, 1, v[96:97]\n"\
      "v_mad_u64_u32 v[112:113], s[44:45], -1, 1, v[108:109]\n"\
      "s_or_b64 s[38:39], s[38:39], s[36:37]\n"\
      "v_cndmask_b32_e64 v104, v96, v100, s[38:39]\n"\
      "s_or_b64 s[44:45], s[44:45], s[42:43]\n"\
      "v_cndmask_b32_e64 v116, v108, v112, s[44:45]\n"\
      "v_cndmask_b32_e64 v105, v97, v101, s[38:39]\n"\
      "v_add_co_u32_e64 v96, s[40:41], v36, v104\n"\
      "v_cndmask_b32_e64 v39, v39, v63, s[20:21]\n"\
      "v_cndmask_b32_e64 v117, v109, v113, s[44:45]\n"\
      "v_add_co_u32_e64 v108, s[46:47], v38, v116\n"\
      "v_addc_co_u32_e64 v97, s[40:41], v37, v105, s[40:41]\n"\
      "v_sub_co_u32_e64 v92, s[36:37], v36, v104\n"\
      "v_addc_co_u32_e64 v109, s[46:47], v39, v117, s[46:47]\n"\
      "v_sub_co_u32_e64 v94, s[42:43], v38, v116\n"\
      "v_subb_co_u32_e64 v93, s[38:39], v37, v105, s[36:37]\n"\
      "v_cndmask_b32_e64 v101, 0, -1, s[40:41]\n"\
      "v_subb_co_u32_e64 v95, s[44:45], v39, v117, s[42:43]\n"\
      "v_cndmask_b32_e64 v113, 0, -1, s[46:47]\n"\
      "v_cndmask_b32_e64 v100, 0, -1, s[38:39]\n"\
      "v_addc_co_u32_e64 v92, s[36:37], v92, 0, s[38:39]\n"\
      "v_mad_u64_u32 v[36:37], s[24:25], v101, 1, v[96:97]\n"\
      "v_cndmask_b32_e64 v112, 0, -1, s[44:45]\n"\
      "v_addc_co_u32_e64 v94, s[42:43], v94, 0, s[44:45]\n"\
      "v_mad_u64_u32 v[38:39], s[24:25], v113, 1, v[108:109]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[36:37]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[38:39]\n"\
      "v_addc_co_u32_e64 v93, s[24:25], v93, v100, s[36:37]\n"\
      "v_cndmask_b32_e64 v36, v36, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v37, v37, v97, s[38:39]\n"\
      "v_addc_co_u32_e64 v95, s[24:25], v95, v112, s[42:43]\n"\
      "v_cndmask_b32_e64 v38, v38, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v39, v39, v109, s[44:45]\n"\
      "v_mad_u64_u32 v[96:97], s[38:39], -1, 1, v[92:93]\n"\
      "v_mad_u64_u32 v[108:109], s[44:45], -1, 1, v[94:95]\n"\
      "s_nop 0\n"\
      "v_cndmask_b32_e64 v92, v92, v96, s[38:39]\n"\
      "v_cndmask_b32_e64 v93, v93, v97, s[38:39]\n"\
      "v_cndmask_b32_e64 v94, v94, v108, s[44:45]\n"\
      "v_cndmask_b32_e64 v95, v95, v109, s[44:45]\n"\
      "global_store_dwordx2 %[l8], v[8:9], s[78:79] offset:0\n"\
      "global_store_dwordx2 %[l8], v[10:11], s[78:79] offset:512\n"\
      "global_store_dwordx2 %[l8], v[12:13], s[78:79] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[14:15], s[78:79] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[16:17], s[78:79] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[18:19], s[78:79] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[20:21], s[78:79] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[22:23], s[78:79] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[24:25], s[80:81] offset:0\n"\
      "global_store_dwordx2 %[l8], v[26:27], s[80:81] offset:512\n"\
      "global_store_dwordx2 %[l8], v[28:29], s[80:81] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[30:31], s[80:81] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[32:33], s[80:81] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[34:35], s[80:81] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[36:37], s[80:81] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[38:39], s[80:81] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[64:65], s[82:83] offset:0\n"\
      "global_store_dwordx2 %[l8], v[66:67], s[82:83] offset:512\n"\
      "global_store_dwordx2 %[l8], v[68:69], s[82:83] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[70:71], s[82:83] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[72:73], s[82:83] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[74:75], s[82:83] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[76:77], s[82:83] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[78:79], s[82:83] offset:3584\n"\
      "global_store_dwordx2 %[l8], v[80:81], s[84:85] offset:0\n"\
      "global_store_dwordx2 %[l8], v[82:83], s[84:85] offset:512\n"\
      "global_store_dwordx2 %[l8], v[84:85], s[84:85] offset:1024\n"\
      "global_store_dwordx2 %[l8], v[86:87], s[84:85] offset:1536\n"\
      "global_store_dwordx2 %[l8], v[88:89], s[84:85] offset:2048\n"\
      "global_store_dwordx2 %[l8], v[90:91], s[84:85] offset:2560\n"\
      "global_store_dwordx2 %[l8], v[92:93], s[84:85] offset:3072\n"\
      "global_store_dwordx2 %[l8], v[94:95], s[84:85] offset:3584\n"\
      "s_waitcnt vmcnt(0)\n"\
      :: __VA_ARGS__ \
      : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "scc", "memory")


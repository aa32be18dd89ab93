set -e
timeout -k 10 300 python -u tools/dbg/rel_big_dbg.py full_rel_big att_syb.dec_vanilla_attention_3.V_proj.0.weight att_syb.enc_feed_forward_0.conv1.0.weight > gpurun_out/rel_big_dbg.log 2>&1
SAVQA_ATTN_FLASH=1 timeout -k 10 300 python -u tools/dbg/rel_big_dbg.py full_rel_sn > gpurun_out/rel_sn_flash.log 2>&1
SAVQA_ATTN_FLASH=1 timeout -k 10 300 python -u tools/dbg/rel_big_dbg.py full_rel_b2 > gpurun_out/rel_b2_flash.log 2>&1
grep -v amdgpu.ids gpurun_out/rel_big_dbg.log | head -40
grep -v amdgpu.ids gpurun_out/rel_sn_flash.log | head -12
grep -v amdgpu.ids gpurun_out/rel_b2_flash.log | head -12

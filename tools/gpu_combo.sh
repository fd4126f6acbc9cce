bash tools/gpu_r3.sh && bash tools/gpu_sim_world.sh

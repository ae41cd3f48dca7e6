"""indoor-nerf_amd: MI355X-native render_rays path of ryanjsuh/indoor-nerf. Import as `indoor_nerf_amd`
(see ../indoor_nerf_amd.py)."""

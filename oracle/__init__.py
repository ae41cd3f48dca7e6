"""Test infrastructure: CPU oracle of the reference's render_rays path (see nerf_oracle.py)."""

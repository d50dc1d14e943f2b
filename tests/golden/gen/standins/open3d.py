"""open3d stand-in (FIXTURE-GENERATION ONLY): visualisation is not exercised."""

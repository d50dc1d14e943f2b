"""pyrenderer_amd — MI355X-native path-tracing core behind pyrenderer's API."""

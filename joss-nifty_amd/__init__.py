"""nifty_amd: MI355X-native geoVI/MGVI sampling hot path (NIFTy 8.5 API)."""

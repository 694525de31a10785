"""Reference apps on GPU ranks (the native CPU apps are csrc/apps/*.cc)."""

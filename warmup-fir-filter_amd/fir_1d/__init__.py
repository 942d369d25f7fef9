"""MI355X-native mirror of the reference package of the same name."""

print("preparing data")
